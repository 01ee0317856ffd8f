"""OpenAI-compatible HTTP server (SURVEY.md G4, H2/H3 integration, §5.5 metrics).

Reference: ``Scripts/inference/07-deepseek1.5b-api-infr.py`` — FastAPI ``POST /v1/chat/completions``
with Pydantic request/response models, ``chatcmpl-<uuid>`` ids, a system message prepended, and
``stream=True`` answered with 501.  This server implements the same schema plus:

* ``stream=True`` as Server-Sent Events (``chat.completion.chunk`` deltas, ``data: [DONE]``);
* ``POST /v1/completions``, ``GET /v1/models``, ``GET /health`` (k8s probes), ``GET /metrics``
  (Prometheus text: ``lipa_num_requests_waiting`` etc., the KEDA trigger of
  ``05-KEDA-AutoScale/keda-scaledobject.yaml``);
* optional pre-call moderation (LiteLLM ``guardrails: openai_moderation pre_call``,
  ``litellm-config-with-guard-model.yaml:24-33``): flagged input → HTTP 400 with the moderation
  result;
* optional ``X-API-KEY`` / ``Authorization: Bearer`` auth.

Generation runs on the :class:`~llm_in_practise_amd.infer.engine.ServingEngine` worker
(continuous batching: requests join and leave the running decode batch every iteration).
"""
from __future__ import annotations

import asyncio
import json
import time
import uuid
from typing import Literal, Optional, Union

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse
from pydantic import BaseModel, Field

from .engine import SamplingParams, ServingEngine


class ChatMessage(BaseModel):
    role: Literal["system", "user", "assistant"]
    content: str


class ChatCompletionRequest(BaseModel):
    model: Optional[str] = None
    messages: list[ChatMessage]
    temperature: float = Field(0.7, ge=0.0, le=2.0)
    top_p: float = Field(1.0, gt=0.0, le=1.0)
    top_k: int = Field(0, ge=0)
    repetition_penalty: float = Field(1.0, gt=0.0)
    max_tokens: int = Field(256, ge=1, le=32768)
    stream: bool = False
    stop: Optional[Union[str, list[str]]] = None
    ignore_eos: bool = False


class CompletionRequest(BaseModel):
    model: Optional[str] = None
    prompt: str
    temperature: float = Field(0.7, ge=0.0, le=2.0)
    top_p: float = Field(1.0, gt=0.0, le=1.0)
    top_k: int = Field(0, ge=0)
    repetition_penalty: float = Field(1.0, gt=0.0)
    max_tokens: int = Field(256, ge=1, le=32768)
    stream: bool = False
    stop: Optional[Union[str, list[str]]] = None
    ignore_eos: bool = False


class ChoiceMessage(BaseModel):
    role: str = "assistant"
    content: str


class Choice(BaseModel):
    index: int
    message: ChoiceMessage
    finish_reason: str


class Usage(BaseModel):
    prompt_tokens: int
    completion_tokens: int
    total_tokens: int


class ChatCompletionResponse(BaseModel):
    id: str
    object: str = "chat.completion"
    created: int
    model: str
    choices: list[Choice]
    usage: Usage


def _params(req) -> SamplingParams:
    stop = [req.stop] if isinstance(req.stop, str) else req.stop
    return SamplingParams(max_tokens=req.max_tokens, temperature=req.temperature, top_p=req.top_p, top_k=req.top_k,
                          repetition_penalty=req.repetition_penalty, stop=stop,
                          ignore_eos=req.ignore_eos)


def create_app(engine: ServingEngine, api_key: str | None = None, moderation=None) -> FastAPI:
    """``moderation``: optional callable ``text -> dict`` (OpenAI moderation response), e.g.
    :meth:`llm_in_practise_amd.infer.guard.GuardClient.moderate_sync`."""
    app = FastAPI(title="llm_in_practise_amd OpenAI-compatible server")

    @app.middleware("http")
    async def auth(request: Request, call_next):
        if api_key and request.url.path.startswith("/v1"):
            key = request.headers.get("X-API-KEY") or request.headers.get("Authorization", "").removeprefix(
                "Bearer ").strip()
            if key != api_key:
                return JSONResponse(status_code=401, content={"error": "Unauthorized"})
        return await call_next(request)

    async def _moderate(text: str):
        if moderation is None:
            return
        res = await asyncio.to_thread(moderation, text)
        if res["results"][0]["flagged"]:
            raise HTTPException(status_code=400, detail={"error": "content_policy_violation", "moderation": res})

    @app.get("/ui")
    async def ui():
        """Browser chat page (the Gradio web UI of ``Scripts/inference/06-*webui*.py`` as plain
        HTML + SSE: streamed deltas, temperature / top-p sliders, multi-turn history)."""
        from fastapi.responses import HTMLResponse
        return HTMLResponse(_UI_HTML.replace("__MODEL__", engine.model_name))

    @app.get("/health")
    async def health():
        return {"status": "ok", "model": engine.model_name}

    @app.get("/v1/models")
    async def models():
        names = getattr(engine, "served_models", None) or [engine.model_name]
        return {"object": "list", "data": [{"id": n, "object": "model", "created": int(time.time()),
                                            "owned_by": "llm_in_practise_amd",
                                            **({"parent": engine.model_name} if n != engine.model_name else {})}
                                           for n in names]}

    def _target(model):
        """Multi-LoRA serving (vLLM --lora-modules): the request's ``model`` picks the adapter;
        with adapters loaded an unknown name is a 404, without any every name maps to the base."""
        if getattr(engine, "mlora", None) is None:
            return None
        if model is None or model in engine.served_models:
            return model
        raise HTTPException(status_code=404, detail=f"The model `{model}` does not exist.")

    @app.get("/metrics")
    async def metrics():
        return PlainTextResponse(engine.prometheus(), media_type="text/plain; version=0.0.4")

    @app.post("/v1/chat/completions")
    async def chat(req: ChatCompletionRequest):
        msgs = [m.model_dump() for m in req.messages]
        await _moderate("\n".join(m["content"] for m in msgs if m["role"] == "user"))
        prompt = engine.build_chat_prompt(msgs)
        cid, created = "chatcmpl-" + uuid.uuid4().hex, int(time.time())
        name = req.model or engine.model_name
        tgt = _target(req.model)
        if req.stream:
            return StreamingResponse(_sse_chat(engine, prompt, _params(req), cid, created, name, tgt),
                                     media_type="text/event-stream")
        res = await asyncio.to_thread(_complete, engine, prompt, _params(req), tgt)
        return ChatCompletionResponse(
            id=cid, created=created, model=name,
            choices=[Choice(index=0, message=ChoiceMessage(content=res["text"]), finish_reason=res["finish_reason"])],
            usage=Usage(prompt_tokens=res["prompt_tokens"], completion_tokens=res["completion_tokens"],
                        total_tokens=res["prompt_tokens"] + res["completion_tokens"]))

    @app.post("/v1/completions")
    async def completions(req: CompletionRequest):
        await _moderate(req.prompt)
        cid, created = "cmpl-" + uuid.uuid4().hex, int(time.time())
        name = req.model or engine.model_name
        tgt = _target(req.model)
        if req.stream:
            return StreamingResponse(_sse_completion(engine, req.prompt, _params(req), cid, created, name, tgt),
                                     media_type="text/event-stream")
        res = await asyncio.to_thread(_complete, engine, req.prompt, _params(req), tgt)
        return {"id": cid, "object": "text_completion", "created": created, "model": name,
                "choices": [{"index": 0, "text": res["text"], "finish_reason": res["finish_reason"],
                             "logprobs": None}],
                "usage": {"prompt_tokens": res["prompt_tokens"], "completion_tokens": res["completion_tokens"],
                          "total_tokens": res["prompt_tokens"] + res["completion_tokens"]}}

    return app


def _complete(engine, prompt, params, model=None):
    return engine.complete(prompt, params, model=model) if model is not None else engine.complete(prompt, params)


async def _aiter_stream(engine, prompt, params, model=None):
    from .engine import AsyncOut
    from .mp_engine import EngineClient
    if not isinstance(engine, (ServingEngine, EngineClient)):
        it = engine.stream(prompt, params, model=model) if model is not None else engine.stream(prompt, params)
        while True:
            item = await asyncio.to_thread(next, it, None)
            if item is None:
                return
            yield item
        return
    out = AsyncOut()
    engine.submit(prompt, params, stream=True, model=model, out=out)
    while True:
        kind, val = await out.get()
        if kind == "delta":
            yield val, None
        elif kind == "final":
            yield "", val
            return
        else:
            raise RuntimeError(val)


async def _sse_chat(engine, prompt, params, cid, created, name, model=None):
    head = {"id": cid, "object": "chat.completion.chunk", "created": created, "model": name}
    yield "data: " + json.dumps({**head, "choices": [{"index": 0, "delta": {"role": "assistant"},
                                                      "finish_reason": None}]}) + "\n\n"
    async for delta, final in _aiter_stream(engine, prompt, params, model):
        if final is None:
            yield "data: " + json.dumps({**head, "choices": [{"index": 0, "delta": {"content": delta},
                                                              "finish_reason": None}]}, ensure_ascii=False) + "\n\n"
        else:
            yield "data: " + json.dumps({**head, "choices": [{"index": 0, "delta": {},
                                                              "finish_reason": final["finish_reason"]}]}) + "\n\n"
    yield "data: [DONE]\n\n"


async def _sse_completion(engine, prompt, params, cid, created, name, model=None):
    head = {"id": cid, "object": "text_completion", "created": created, "model": name}
    async for delta, final in _aiter_stream(engine, prompt, params, model):
        fr = None if final is None else final["finish_reason"]
        yield "data: " + json.dumps({**head, "choices": [{"index": 0, "text": delta, "finish_reason": fr}]},
                                    ensure_ascii=False) + "\n\n"
    yield "data: [DONE]\n\n"


_UI_HTML = """<!doctype html><html><head><meta charset="utf-8"><title>__MODEL__</title>
<style>body{font-family:sans-serif;max-width:860px;margin:2em auto}#log div{margin:.4em 0;white-space:pre-wrap}
.u{color:#036}.a{color:#222}textarea{width:100%;height:4em}</style></head><body>
<h3>__MODEL__</h3><div id="log"></div><textarea id="q"></textarea><br>
temperature <input id="t" type="range" min="0" max="1.5" step="0.05" value="0.7"><span id="tv">0.7</span>
top-p <input id="p" type="range" min="0.05" max="1" step="0.05" value="0.9"><span id="pv">0.9</span>
<button onclick="send()">send</button> <button onclick="hist=[];log.innerHTML=''">clear</button>
<script>
let hist=[];const log=document.getElementById('log');
for(const [s,v] of [['t','tv'],['p','pv']]){const e=document.getElementById(s);e.oninput=()=>document.getElementById(v).textContent=e.value;}
async function send(){const q=document.getElementById('q').value;if(!q)return;document.getElementById('q').value='';
hist.push({role:'user',content:q});const u=document.createElement('div');u.className='u';u.textContent='user: '+q;log.appendChild(u);
const a=document.createElement('div');a.className='a';a.textContent='assistant: ';log.appendChild(a);
const r=await fetch('/v1/chat/completions',{method:'POST',headers:{'Content-Type':'application/json'},
body:JSON.stringify({messages:hist,stream:true,max_tokens:512,temperature:+document.getElementById('t').value,top_p:+document.getElementById('p').value})});
const rd=r.body.getReader();const dec=new TextDecoder();let buf='',text='';
while(true){const {done,value}=await rd.read();if(done)break;buf+=dec.decode(value,{stream:true});
let i;while((i=buf.indexOf('\\n\\n'))>=0){const line=buf.slice(0,i);buf=buf.slice(i+2);
if(!line.startsWith('data: ')||line==='data: [DONE]')continue;const d=JSON.parse(line.slice(6)).choices[0].delta||{};
if(d.content){text+=d.content;a.textContent='assistant: '+text;}}}
hist.push({role:'assistant',content:text});}
</script></body></html>"""


def serve(engine: ServingEngine, host: str = "0.0.0.0", port: int = 8000, log_level: str = "info", **kw):
    import uvicorn
    uvicorn.run(create_app(engine, **kw), host=host, port=port, log_level=log_level)
