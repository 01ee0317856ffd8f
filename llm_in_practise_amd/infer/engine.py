"""Serving engine: model + tokenizer + a dynamic-batching worker.

The reference serves through vLLM; its own FastAPI app (``Scripts/inference/07-…-api-infr.py``)
runs one ``model.generate`` per request.  Here one worker thread owns the GPU and drains a
request queue: requests that arrive while a batch is running are grouped (up to
``max_batch``) by identical sampling parameters and decoded TOGETHER — right-padded prompts of
different lengths, per-row KV positions (``infer/generate.py``) — so concurrent clients share
every decode step (the weights are read once per step for the whole batch, which is what makes
decode on a 288 GB HBM part efficient).  Streaming requests get per-row text deltas through a
fan-out streamer.  Metrics for ``/metrics`` (Prometheus text) are kept here.
"""
from __future__ import annotations

import dataclasses
import queue
import threading
import time
import uuid
from typing import Any

import torch

from ..train.data import render_chatml
from .generate import generate


@dataclasses.dataclass
class SamplingParams:
    max_tokens: int = 256
    temperature: float = 0.7
    top_p: float = 1.0
    top_k: int = 0
    repetition_penalty: float = 1.0
    stop: list[str] | None = None

    def key(self):
        return (self.temperature, self.top_p, self.top_k, self.repetition_penalty)


@dataclasses.dataclass
class _Request:
    prompt_ids: list[int]
    params: SamplingParams
    stream: bool
    out: "queue.Queue[Any]"
    t_arrive: float
    rid: str = dataclasses.field(default_factory=lambda: uuid.uuid4().hex)


class _Histogram:
    def __init__(self, buckets):
        self.buckets = list(buckets)
        self.counts = [0] * (len(self.buckets) + 1)
        self.sum = 0.0
        self.n = 0

    def observe(self, v):
        self.sum += v
        self.n += 1
        for i, b in enumerate(self.buckets):
            if v <= b:
                self.counts[i] += 1
        self.counts[-1] += 1

    def render(self, name):
        lines = [f"# TYPE {name} histogram"]
        for b, c in zip(self.buckets, self.counts):
            lines.append(f'{name}_bucket{{le="{b}"}} {c}')
        lines += [f'{name}_bucket{{le="+Inf"}} {self.counts[-1]}', f"{name}_sum {self.sum}", f"{name}_count {self.n}"]
        return lines


class _FanoutStreamer:
    """Per-row incremental detokenisation for a batched decode."""

    def __init__(self, tokenizer, reqs: list[_Request], eos: set[int]):
        self.tok, self.reqs, self.eos = tokenizer, reqs, eos
        self.ids = [[] for _ in reqs]
        self.sent = [0] * len(reqs)
        self.done = [False] * len(reqs)
        self.first = [None] * len(reqs)

    def put(self, tok: torch.Tensor):
        now = time.time()
        for i, t in enumerate(tok.tolist()):
            if self.done[i]:
                continue
            if self.first[i] is None:
                self.first[i] = now
            if t in self.eos or len(self.ids[i]) >= self.reqs[i].params.max_tokens:
                self.done[i] = True
                continue
            self.ids[i].append(t)
            if self.reqs[i].stream:
                text = self.tok.decode(self.ids[i], skip_special_tokens=True)
                if len(text) > self.sent[i] and not text.endswith("�"):
                    self.reqs[i].out.put(("delta", text[self.sent[i]:]))
                    self.sent[i] = len(text)

    def end(self):
        pass


class ServingEngine:
    def __init__(self, model, tokenizer, model_name: str = "lipa-model", max_batch: int = 16,
                 system_prompt: str | None = None, chat_template: str = "auto", space_before_end: bool = False):
        self.model, self.tok, self.model_name = model, tokenizer, model_name
        self.max_batch = max_batch
        self.system_prompt = system_prompt
        self.chat_template = chat_template
        self.space_before_end = space_before_end
        self.device = next(model.parameters()).device
        eos = getattr(tokenizer, "eos_token_id", None)
        self.eos = {eos} if isinstance(eos, int) else set(eos or [])
        im_end = None
        if hasattr(tokenizer, "convert_tokens_to_ids"):
            try:
                im_end = tokenizer.convert_tokens_to_ids("<|im_end|>")
            except Exception:
                im_end = None
        if isinstance(im_end, int) and im_end >= 0 and im_end != getattr(tokenizer, "unk_token_id", None):
            self.eos.add(im_end)
        self.pad = getattr(tokenizer, "pad_token_id", None)
        if self.pad is None:
            self.pad = next(iter(self.eos), 0)
        self.q: "queue.Queue[_Request]" = queue.Queue()
        self.lock = threading.Lock()
        self.stats = {"requests_total": 0, "prompt_tokens_total": 0, "generation_tokens_total": 0,
                      "batches_total": 0, "running": 0}
        self.h_latency = _Histogram([0.05, 0.1, 0.25, 0.5, 1, 2, 5, 10, 30, 60])
        self.h_ttft = _Histogram([0.01, 0.025, 0.05, 0.1, 0.2, 0.5, 1, 2, 5])
        self._stop = False
        self._worker = threading.Thread(target=self._loop, daemon=True)
        self._worker.start()

    # ------------------------------------------------------------------ prompt formatting
    def build_chat_prompt(self, messages: list[dict]) -> str:
        msgs = list(messages)
        if self.system_prompt and not any(m.get("role") == "system" for m in msgs):
            msgs.insert(0, {"role": "system", "content": self.system_prompt})     # G4 prepends a system msg
        if self.chat_template == "auto" and hasattr(self.tok, "apply_chat_template") and \
                getattr(self.tok, "chat_template", None):
            return self.tok.apply_chat_template(msgs, tokenize=False, add_generation_prompt=True)
        return render_chatml(msgs, space_before_end=self.space_before_end, add_generation_prompt=True)

    def encode(self, text: str) -> list[int]:
        return list(self.tok.encode(text, add_special_tokens=False))

    # ------------------------------------------------------------------ request API (thread-safe)
    def submit(self, prompt: str, params: SamplingParams, stream: bool = False) -> _Request:
        ids = self.encode(prompt)
        r = _Request(ids, params, stream, queue.Queue(), time.time())
        self.q.put(r)
        return r

    def complete(self, prompt: str, params: SamplingParams, timeout: float | None = None) -> dict:
        r = self.submit(prompt, params, stream=False)
        while True:
            kind, val = r.out.get(timeout=timeout)
            if kind == "final":
                return val
            if kind == "error":
                raise RuntimeError(val)

    def stream(self, prompt: str, params: SamplingParams, timeout: float | None = None):
        r = self.submit(prompt, params, stream=True)
        while True:
            kind, val = r.out.get(timeout=timeout)
            if kind == "delta":
                yield val, None
            elif kind == "final":
                yield "", val
                return
            elif kind == "error":
                raise RuntimeError(val)

    def shutdown(self):
        self._stop = True

    # ------------------------------------------------------------------ worker
    def _collect(self) -> list[_Request]:
        first = self.q.get()
        batch = [first]
        pending = []
        while len(batch) < self.max_batch:
            try:
                r = self.q.get_nowait()
            except queue.Empty:
                break
            (batch if r.params.key() == first.params.key() else pending).append(r)
        for r in pending:
            self.q.put(r)
        return batch

    def _loop(self):
        while not self._stop:
            batch = self._collect()
            try:
                self._run(batch)
            except Exception as e:  # report to every waiting client, keep serving
                for r in batch:
                    r.out.put(("error", repr(e)))

    def _run(self, batch: list[_Request]):
        B = len(batch)
        S = max(len(r.prompt_ids) for r in batch)
        ids = torch.full((B, S), self.pad, dtype=torch.long)
        am = torch.zeros(B, S, dtype=torch.long)
        for i, r in enumerate(batch):
            ids[i, :len(r.prompt_ids)] = torch.tensor(r.prompt_ids, dtype=torch.long)
            am[i, :len(r.prompt_ids)] = 1
        p = batch[0].params
        max_new = max(r.params.max_tokens for r in batch)
        fan = _FanoutStreamer(self.tok, batch, self.eos)
        self.stats["running"] = B
        t0 = time.time()
        with self.lock:
            out = generate(self.model, ids.to(self.device), am.to(self.device), max_new_tokens=max_new,
                           do_sample=p.temperature > 0, temperature=p.temperature, top_p=p.top_p, top_k=p.top_k,
                           repetition_penalty=p.repetition_penalty, eos_token_id=sorted(self.eos) or None,
                           pad_token_id=self.pad, streamer=fan)
        self.stats["running"] = 0
        self.stats["batches_total"] += 1
        t1 = time.time()
        for i, r in enumerate(batch):
            gen = fan.ids[i][:r.params.max_tokens]
            text = self.tok.decode(gen, skip_special_tokens=True)
            finish = "stop" if fan.done[i] and len(gen) < r.params.max_tokens else "length"
            if r.params.stop:
                cut = min((text.find(s) for s in r.params.stop if s and s in text), default=-1)
                if cut >= 0:
                    text, finish = text[:cut], "stop"
            self.stats["requests_total"] += 1
            self.stats["prompt_tokens_total"] += len(r.prompt_ids)
            self.stats["generation_tokens_total"] += len(gen)
            self.h_latency.observe(t1 - r.t_arrive)
            if fan.first[i] is not None:
                self.h_ttft.observe(fan.first[i] - r.t_arrive)
            r.out.put(("final", {"text": text, "finish_reason": finish, "prompt_tokens": len(r.prompt_ids),
                                 "completion_tokens": len(gen), "latency_s": t1 - r.t_arrive,
                                 "batch_size": B, "decode_s": t1 - t0}))

    # ------------------------------------------------------------------ metrics
    def prometheus(self) -> str:
        s = self.stats
        lines = [
            "# TYPE lipa_requests_total counter", f"lipa_requests_total {s['requests_total']}",
            "# TYPE lipa_prompt_tokens_total counter", f"lipa_prompt_tokens_total {s['prompt_tokens_total']}",
            "# TYPE lipa_generation_tokens_total counter",
            f"lipa_generation_tokens_total {s['generation_tokens_total']}",
            "# TYPE lipa_batches_total counter", f"lipa_batches_total {s['batches_total']}",
            "# TYPE lipa_num_requests_waiting gauge", f"lipa_num_requests_waiting {self.q.qsize()}",
            "# TYPE lipa_num_requests_running gauge", f"lipa_num_requests_running {s['running']}",
        ]
        lines += self.h_latency.render("lipa_e2e_request_latency_seconds")
        lines += self.h_ttft.render("lipa_time_to_first_token_seconds")
        if torch.cuda.is_available():
            lines += ["# TYPE lipa_hbm_allocated_bytes gauge",
                      f"lipa_hbm_allocated_bytes {torch.cuda.memory_allocated()}"]
        return "\n".join(lines) + "\n"
