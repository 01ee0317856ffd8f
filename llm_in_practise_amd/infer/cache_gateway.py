"""L2 / L3 response-cache gateway in front of OpenAI-compatible backends.

Reference: the Flask gateway embedded in ``LLM_on_Kubernetes/Inference_Platfrom/README.md:3041-3144``:
an **exact** cache keyed by SHA-256 of the request (TTL 300 s) and a **"semantic"** cache keyed
by SHA-256 of the first 8 embedding dimensions rounded to 2 decimals (TTL 600 s), both in
Redis, with Prometheus hit/miss counters, proxying misses to vLLM.

Here: a FastAPI app with the same two levels and key rules.  Storage is a pluggable TTL store —
in-process (default, LRU-bounded) or Redis when a ``redis://`` URL is given and the ``redis``
package is importable.  The "semantic" embedding is a deterministic feature-hashing bag of
word/character n-grams (the reference does not pin an embedding model; any callable
``text -> list[float]`` can be passed).  Only non-streaming, greedy-or-seeded requests are
cacheable by default (``temperature == 0``), as sampling would otherwise return a stale draw.
"""
from __future__ import annotations

import collections
import hashlib
import json
import math
import re
import threading
import time
from typing import Callable

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse


class TTLStore:
    """Thread-safe in-process key → (expiry, value) store with LRU bound."""

    def __init__(self, max_items: int = 10000):
        self.max_items = max_items
        self._d: "collections.OrderedDict[str, tuple[float, str]]" = collections.OrderedDict()
        self._lock = threading.Lock()

    def get(self, key: str):
        with self._lock:
            item = self._d.get(key)
            if item is None:
                return None
            if item[0] < time.time():
                del self._d[key]
                return None
            self._d.move_to_end(key)
            return item[1]

    def setex(self, key: str, ttl: int, value: str):
        with self._lock:
            self._d[key] = (time.time() + ttl, value)
            self._d.move_to_end(key)
            while len(self._d) > self.max_items:
                self._d.popitem(last=False)


def make_store(url: str | None):
    if url and url.startswith("redis://"):
        import redis  # optional dependency
        return redis.Redis.from_url(url, decode_responses=True)
    return TTLStore()


def hashing_embedding(text: str, dim: int = 256) -> list[float]:
    """L2-normalised feature-hashing embedding of lower-cased words and character 3-grams."""
    v = [0.0] * dim
    t = text.lower()
    feats = re.findall(r"\w+", t) + [t[i:i + 3] for i in range(max(0, len(t) - 2))]
    for f in feats:
        h = int.from_bytes(hashlib.blake2b(f.encode(), digest_size=8).digest(), "little")
        v[h % dim] += 1.0 if (h >> 63) & 1 else -1.0
    n = math.sqrt(sum(x * x for x in v)) or 1.0
    return [x / n for x in v]


def exact_key(body: dict) -> str:
    return "exact:" + hashlib.sha256(json.dumps(body, sort_keys=True, ensure_ascii=False).encode()).hexdigest()


def semantic_key(body: dict, embed: Callable[[str], list[float]]) -> str:
    text = "\n".join(m.get("content", "") for m in body.get("messages", [])) or body.get("prompt", "")
    head = [round(x, 2) for x in embed(text)[:8]]       # the reference's 8-dim / 2-decimal rule
    return "semantic:" + hashlib.sha256((body.get("model", "") + json.dumps(head)).encode()).hexdigest()


def create_cache_gateway(backend: Callable[[str, dict], dict], store=None, exact_ttl: int = 300,
                         semantic_ttl: int = 600, embed: Callable[[str], list[float]] = hashing_embedding,
                         cache_sampled: bool = False) -> FastAPI:
    """``backend(path, body) -> response dict`` performs the upstream call (see :func:`http_backend`)."""
    store = store if store is not None else TTLStore()
    app = FastAPI(title="lipa cache gateway")
    counters = collections.Counter()

    def cacheable(body: dict) -> bool:
        return not body.get("stream") and (cache_sampled or float(body.get("temperature", 1.0)) == 0.0)

    async def handle(path: str, request: Request):
        body = await request.json()
        counters["requests_total"] += 1
        if not cacheable(body):
            counters["bypass_total"] += 1
            return JSONResponse(backend(path, body))
        ek, sk = exact_key({"path": path, **body}), semantic_key(body, embed)
        for level, key in (("exact", ek), ("semantic", sk)):
            hit = store.get(key)
            if hit is not None:
                counters[f"hits_{level}_total"] += 1
                resp = json.loads(hit)
                resp.setdefault("lipa_cache", level)
                return JSONResponse(resp)
        counters["misses_total"] += 1
        resp = backend(path, body)
        payload = json.dumps(resp, ensure_ascii=False)
        store.setex(ek, exact_ttl, payload)
        store.setex(sk, semantic_ttl, payload)
        return JSONResponse(resp)

    @app.post("/v1/chat/completions")
    async def chat(request: Request):
        return await handle("/v1/chat/completions", request)

    @app.post("/v1/completions")
    async def completions(request: Request):
        return await handle("/v1/completions", request)

    @app.get("/health")
    async def health():
        return {"status": "ok"}

    @app.get("/metrics")
    async def metrics():
        lines = []
        for name in ("requests_total", "bypass_total", "misses_total", "hits_exact_total", "hits_semantic_total"):
            lines += [f"# TYPE lipa_cache_{name} counter", f"lipa_cache_{name} {counters[name]}"]
        return PlainTextResponse("\n".join(lines) + "\n")

    return app


def http_backend(base_url: str, api_key: str | None = None, timeout: float = 600.0):
    """Upstream caller for :func:`create_cache_gateway` (any OpenAI-compatible server)."""
    import httpx
    client = httpx.Client(base_url=base_url.rstrip("/"), timeout=timeout)
    headers = {"Authorization": f"Bearer {api_key}"} if api_key else {}

    def call(path: str, body: dict) -> dict:
        r = client.post(path, json=body, headers=headers)
        r.raise_for_status()
        return r.json()
    return call
