"""Safety-moderation adapter: a Llama-Guard-style classifier exposed through the
OpenAI ``/v1/moderations`` schema so a gateway (LiteLLM ``openai_moderation`` guardrail) or our
own server can pre-screen prompts.

Behaviour mirrors ``Deployment/litellm-proxy/llama-guard-wrapper``: a JSON-only classification
prompt (safe / S-code categories / explanation) sent to a completions backend
(``model_client.py:18-32``) with retries and linear backoff (``:35-58``); a JSON answer is
preferred, else the native ``safe|unsafe\\nS1 S4`` form is parsed (``:69-85``) and keyword
heuristics add S11 / S9 / S10 (``:87-128``); S1..S14 map onto the OpenAI categories
(``openai_moderation_map.py:11-64``); optional ``X-API-KEY`` auth (``app.py:22-31``).

The backend is pluggable: an HTTP ``/v1/completions`` URL (e.g. our own server hosting the guard
model) or any in-process callable ``prompt -> text``.
"""
from __future__ import annotations

import json
import os
import re
import time
import uuid
from typing import Callable, Union

from pydantic import BaseModel


class ModerationRequest(BaseModel):
    input: Union[str, list[str]]


OPENAI_CATEGORIES = ("hate", "hate/threatening", "harassment", "harassment/threatening", "self-harm",
                     "self-harm/intent", "self-harm/instructions", "sexual", "sexual/minors", "violence",
                     "violence/graphic")

# MLCommons hazard taxonomy S-codes (Llama Guard 3) → OpenAI moderation categories
SCODE_TO_OPENAI = {
    "S1": ("violence",), "S2": ("violence",), "S3": ("sexual",), "S4": ("sexual/minors",),
    "S5": ("harassment",), "S6": ("self-harm",), "S7": ("self-harm/intent",), "S8": ("self-harm/instructions",),
    "S9": ("violence",), "S10": ("hate",), "S11": ("self-harm/instructions",), "S12": ("hate/threatening",),
    "S13": ("harassment/threatening",), "S14": ("sexual/minors",),
}

GUARD_SYSTEM = (
    "You are a safety classifier using the S-code hazard taxonomy S1..S14.\n"
    "Reply with JSON only, exactly these keys:\n"
    '  "safe": true|false,\n'
    '  "categories": up to three S-codes ordered by relevance (e.g. ["S11"]),\n'
    '  "explanation": one short sentence.\n'
    "Self-harm or suicide instructions -> S11. Explosives or weapons -> S9 (or S1/S2). "
    "Hate against a protected group -> S10. Output nothing but the JSON object.")

_HEURISTICS = (
    (("suicid", "自杀", "kill myself"), "S11", "keyword heuristic: self-harm"),
    (("bomb", "explosive", "炸弹", "爆炸"), "S9", "keyword heuristic: weapons/explosives"),
    (("racist", "仇恨", "hate them", "杀死他们因为"), "S10", "keyword heuristic: hate speech"),
)


def build_guard_prompt(text: str) -> str:
    """Llama-3 header format used by Llama Guard 3."""
    return ("<|begin_of_text|><|start_header_id|>system<|end_header_id|>\n" + GUARD_SYSTEM + "\n"
            "<|start_header_id|>user<|end_header_id|>\n" + text.strip() + "\n"
            "<|start_header_id|>assistant<|end_header_id|>\n")


def parse_guard_output(out: str, text: str = "") -> dict:
    """JSON answer if present, else native ``safe``/``unsafe`` + S-codes, plus keyword rules."""
    s = (out or "").strip()
    m = re.search(r"\{.*\}", s, re.S)
    if m:
        try:
            d = json.loads(m.group(0))
            cats = [c.upper() for c in (d.get("categories") or []) if isinstance(c, str)]
            return {"safe": bool(d.get("safe", not cats)), "categories": cats,
                    "explanation": str(d.get("explanation", "") or "")}
        except (ValueError, TypeError):
            pass
    lines = [l.strip() for l in s.splitlines() if l.strip()]
    safe = not (lines and "unsafe" in lines[0].lower())
    codes = [c.upper() for c in re.findall(r"[Ss]\d+", " ".join(lines[1:] if len(lines) > 1 else lines))]
    codes = [c for c in codes if c in SCODE_TO_OPENAI]
    res = {"safe": safe, "categories": codes if (codes or safe) else ["UNSPECIFIED"], "explanation": ""}
    low = (text or "").lower()
    for keys, code, why in _HEURISTICS:
        if any(k in low for k in keys):
            if code not in res["categories"]:
                res["categories"].insert(0, code)
            res["safe"] = False
            res["explanation"] = why
            break
    return res


def to_openai_moderation(result: dict, model: str = "llama-guard-3", raw: dict | None = None) -> dict:
    cats = {c: False for c in OPENAI_CATEGORIES}
    scores = {c: 0.0 for c in OPENAI_CATEGORIES}
    for code in result.get("categories", []):
        for c in SCODE_TO_OPENAI.get(code.upper(), ()):
            cats[c] = True
            scores[c] = 1.0
    flagged = not result.get("safe", True)
    return {"id": "modr-" + uuid.uuid4().hex, "model": model,
            "results": [{"flagged": flagged, "categories": cats, "category_scores": scores,
                         "category_applied_input_types": {c: (["text"] if cats[c] else []) for c in cats},
                         "explanation": result.get("explanation", ""), "raw": raw or {}}]}


class GuardClient:
    def __init__(self, backend: str | Callable[[str], str], model: str = "llama-guard-3", retries: int = 2,
                 timeout: float = 30.0, backoff: float = 0.5):
        self.backend, self.model = backend, model
        self.retries, self.timeout, self.backoff = retries, timeout, backoff

    def _complete(self, prompt: str) -> str:
        if callable(self.backend):
            return self.backend(prompt)
        import httpx
        url = self.backend.rstrip("/")
        if not url.endswith("/completions"):
            url += "/v1/completions"
        last = None
        for attempt in range(self.retries + 1):
            try:
                r = httpx.post(url, json={"model": self.model, "prompt": prompt, "max_tokens": 256,
                                          "temperature": 0.0}, timeout=self.timeout)
                if r.status_code != 200:
                    raise RuntimeError(f"guard backend HTTP {r.status_code}: {r.text[:200]}")
                ch = r.json()["choices"][0]
                return ch.get("text") or (ch.get("message") or {}).get("content") or ""
            except (httpx.RequestError,) as e:    # transport errors: retry with linear backoff
                last = e
                time.sleep(self.backoff * (attempt + 1))
        raise RuntimeError(f"guard backend unreachable after {self.retries + 1} attempts: {last}")

    def moderate_sync(self, text: str) -> dict:
        out = self._complete(build_guard_prompt(text))
        return to_openai_moderation(parse_guard_output(out, text), self.model, {"text": out})


def create_guard_app(client: GuardClient, api_key: str | None = None):
    from fastapi import FastAPI, HTTPException, Request
    from fastapi.responses import JSONResponse

    app = FastAPI(title="OpenAI-moderation adapter")
    key = api_key if api_key is not None else os.environ.get("WRAPPER_API_KEY", "")

    @app.middleware("http")
    async def auth(request: Request, call_next):
        if key and request.headers.get("X-API-KEY", "") != key and request.url.path != "/healthz":
            return JSONResponse(status_code=401, content={"error": "Unauthorized"})
        return await call_next(request)

    @app.post("/v1/moderations")
    @app.post("/moderations")
    async def moderations(req: ModerationRequest):
        text = req.input if isinstance(req.input, str) else "\n".join(req.input)
        if not text.strip():
            raise HTTPException(status_code=400, detail="input is required")
        import asyncio
        try:
            return await asyncio.to_thread(client.moderate_sync, text)
        except RuntimeError as e:
            raise HTTPException(status_code=502, detail=str(e))

    @app.get("/healthz")
    async def healthz():
        return {"status": "ok"}

    return app
