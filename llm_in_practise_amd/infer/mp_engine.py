"""Engine core in its own process (vLLM V1 "EngineCore" / frontend-multiprocessing role).

At high concurrency the per-token Python work of an OpenAI server — SSE framing and the event
loop of every open stream — competes for the GIL with the scheduling / detokenising engine
thread, so decode steps that take 12 ms on the GPU at batch 256 were being paced at ~28 ms by
the host (``profiles/serving_*``).  Here the HTTP process only formats and streams; the engine
process owns the GPU, schedules, samples and detokenises, and ships each iteration's outputs
to the frontend as ONE batched message over a pipe:

    frontend (uvicorn + FastAPI)            engine process (GPU)
    EngineClient.submit ──("submit", …)──▶  ServingEngine (its _loop thread)
    receiver thread ◀──[(rid, kind, val)…]── outbox flushed once per engine iteration

The client implements the subset of :class:`~.engine.ServingEngine` the server uses
(``submit`` / ``complete`` / ``stream`` / ``build_chat_prompt`` / ``prometheus`` / names), so
``create_app(EngineClient(...))`` serves exactly like the in-process engine.
"""
from __future__ import annotations

import dataclasses
import multiprocessing as mp
import queue
import threading
import uuid

from .engine import SamplingParams


class _Outbox:
    """Per-request ``out`` inside the engine process: collects (rid, item) for the next flush."""

    def __init__(self, rid: str, sink: list, lock: threading.Lock):
        self.rid, self.sink, self.lock = rid, sink, lock

    def put(self, item):
        with self.lock:
            self.sink.append((self.rid,) + tuple(item))


def _engine_main(factory, factory_args, cmd_conn, out_conn, ready):
    """Child process: build the engine, then serve commands until shutdown."""
    eng = factory(*factory_args)
    sink: list = []
    lock = threading.Lock()
    send_lock = threading.Lock()

    def flush():
        with send_lock:
            with lock:
                if not sink:
                    return
                batch = list(sink)
                sink.clear()
            out_conn.send(batch)

    eng.iteration_hook = flush
    ready.send({"model_name": eng.model_name, "served_models": eng.served_models})
    while True:
        try:
            msg = cmd_conn.recv()
        except EOFError:
            break
        op = msg[0]
        if op == "submit":
            _, rid, prompt, pd, stream, model = msg
            try:
                eng.submit(prompt, SamplingParams(**pd), stream=stream, model=model, out=_Outbox(rid, sink, lock))
            except Exception as e:                # unknown adapter etc.: fail just this request
                with lock:
                    sink.append((rid, "error", repr(e)))
                flush()
        elif op == "metrics":
            with lock:
                sink.append((msg[1], "rpc", eng.prometheus()))
            flush()
        elif op == "shutdown":
            eng.shutdown()
            break
    flush()


def _dispatch(items):
    for q, item in items:
        q.put_nowait(item)


class EngineClient:
    """Frontend-side handle of an engine process (see module docstring).

    ``factory(*args)`` must be a picklable top-level callable returning a ServingEngine; it runs
    in the child (the frontend process never touches the GPU).  ``formatter`` formats chat
    prompts in the frontend (an object with ``build_chat_prompt``, e.g. a ServingEngine-like
    prompt builder over the same tokenizer)."""

    def __init__(self, factory, factory_args: tuple, formatter, start_method: str = "spawn", timeout: float = 1800):
        ctx = mp.get_context(start_method)
        self._cmd_r, self._cmd_w = ctx.Pipe(duplex=False)
        self._out_r, self._out_w = ctx.Pipe(duplex=False)
        rd_r, rd_w = ctx.Pipe(duplex=False)
        self.proc = ctx.Process(target=_engine_main, args=(factory, factory_args, self._cmd_r, self._out_w, rd_w),
                                daemon=True)
        self.proc.start()
        if not rd_r.poll(timeout):
            raise RuntimeError("engine process did not start")
        info = rd_r.recv()
        self.model_name, self.served_models = info["model_name"], info["served_models"]
        self.formatter = formatter
        self._outs: dict[str, object] = {}
        self._send_lock = threading.Lock()
        self._rpc: dict[str, queue.Queue] = {}
        self._rx = threading.Thread(target=self._receive, daemon=True)
        self._rx.start()

    # ---- plumbing ------------------------------------------------------------------------
    def _send(self, msg):
        with self._send_lock:
            self._cmd_w.send(msg)

    def _receive(self):
        while True:
            try:
                batch = self._out_r.recv()
            except (EOFError, OSError):
                for out in list(self._outs.values()):
                    out.put(("error", "engine process exited"))
                return
            by_loop: dict = {}
            for rid, kind, val in batch:
                if kind == "rpc":
                    q = self._rpc.pop(rid, None)
                    if q is not None:
                        q.put(val)
                    continue
                out = self._outs.get(rid)
                if out is None:
                    continue
                loop = getattr(out, "loop", None)
                if loop is not None:           # AsyncOut: one hand-off per event loop per batch
                    by_loop.setdefault(loop, []).append((out.q, (kind, val)))
                else:
                    out.put((kind, val))
                if kind in ("final", "error"):
                    self._outs.pop(rid, None)
            for loop, items in by_loop.items():
                loop.call_soon_threadsafe(_dispatch, items)

    # ---- ServingEngine surface used by infer/server.py -------------------------------------
    @property
    def mlora(self):
        return True if len(self.served_models) > 1 else None

    def build_chat_prompt(self, messages):
        return self.formatter.build_chat_prompt(messages)

    def submit(self, prompt: str, params: SamplingParams, stream: bool = False, model: str | None = None, out=None):
        if model is not None and model not in self.served_models:
            raise KeyError(model)
        rid = uuid.uuid4().hex
        out = out if out is not None else queue.Queue()
        self._outs[rid] = out
        self._send(("submit", rid, prompt, dataclasses.asdict(params), stream, model))
        return out

    def complete(self, prompt: str, params: SamplingParams, timeout: float | None = None, model: str | None = None):
        out = self.submit(prompt, params, stream=False, model=model)
        while True:
            kind, val = out.get(timeout=timeout)
            if kind == "final":
                return val
            if kind == "error":
                raise RuntimeError(val)

    def stream(self, prompt: str, params: SamplingParams, timeout: float | None = None, model: str | None = None):
        out = self.submit(prompt, params, stream=True, model=model)
        while True:
            kind, val = out.get(timeout=timeout)
            if kind == "delta":
                yield val, None
            elif kind == "final":
                yield "", val
                return
            elif kind == "error":
                raise RuntimeError(val)

    def prometheus(self, timeout: float = 10.0) -> str:
        tok = "rpc-" + uuid.uuid4().hex
        q: queue.Queue = queue.Queue()
        self._rpc[tok] = q
        self._send(("metrics", tok))
        return q.get(timeout=timeout)

    def shutdown(self, timeout: float = 30.0):
        try:
            self._send(("shutdown",))
        except (OSError, BrokenPipeError):
            pass
        self.proc.join(timeout)
        if self.proc.is_alive():
            self.proc.terminate()


class PromptFormatter:
    """Chat-prompt formatting in the frontend process (same rules as ServingEngine)."""

    def __init__(self, tokenizer, system_prompt=None, chat_template="auto", space_before_end=False):
        self.tok, self.system_prompt = tokenizer, system_prompt
        self.chat_template, self.space_before_end = chat_template, space_before_end

    def build_chat_prompt(self, messages):
        from .engine import ServingEngine
        return ServingEngine.build_chat_prompt(self, messages)

