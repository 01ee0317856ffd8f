"""Serving engine with iteration-level (continuous) batching.

The reference serves through vLLM (continuous batching, paged KV); its own FastAPI app
(``Scripts/inference/07-…-api-infr.py``) runs one ``model.generate`` per request.  Here one worker
thread owns the GPU and keeps a fixed pool of ``max_batch`` sequence slots over ONE pre-allocated
KV cache ``[max_batch, max_model_len, Hkv·D]`` per layer (288 GB of HBM makes a contiguous cache
per slot affordable: Qwen3-8B, 64 slots × 4096 tokens = 36 GB):

* every iteration, waiting requests are admitted into free slots: their prompts are prefilled
  together (right-padded, fused flash-attention with per-row key lengths) into a scratch cache and
  copied into their slots; their first token is sampled from the prefill logits;
* then ONE decode step runs for all slots at once — each row appends at its own position
  (``KVCache.write_rows``) and the split-K decode-attention kernel reads per-row lengths, so
  sequences of any length and age share every step (weights are read once per step for the
  whole batch);
* finished rows (EOS / max_tokens / cache full) are released immediately and refilled on the next
  iteration — no request waits for another's completion;
* per-request sampling parameters: rows are sampled in groups of identical parameters with the
  fused sampler kernel.

Streaming requests receive text deltas per token; ``/metrics`` data (Prometheus text) is kept here.
"""
from __future__ import annotations

import dataclasses
import queue
import threading
import time
import uuid
from typing import Any

import torch

from ..models.common import KVCache, PackedPrefill
from ..ops.decode import sample
from ..ops.linear import head_logits
from ..train.data import render_chatml


@dataclasses.dataclass
class SamplingParams:
    max_tokens: int = 256
    temperature: float = 0.7
    top_p: float = 1.0
    top_k: int = 0
    repetition_penalty: float = 1.0
    stop: list[str] | None = None
    ignore_eos: bool = False            # vLLM extra param (``vllm bench serve --ignore-eos``)

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
    adapter: int = 0                      # multi-LoRA serving: 0 = base, i = i-th --lora-modules entry


class AsyncOut:
    """Thread-safe ``put`` into an ``asyncio.Queue`` owned by an event loop: the engine thread
    hands each streamed delta to the server's loop with one ``call_soon_threadsafe`` instead of
    the loop polling a ``queue.Queue`` from a worker thread per token."""

    def __init__(self, loop=None):
        import asyncio
        self.loop = loop or asyncio.get_running_loop()
        self.q: "asyncio.Queue" = asyncio.Queue()

    def put(self, item):
        self.loop.call_soon_threadsafe(self.q.put_nowait, item)

    async def get(self):
        return await self.q.get()


class PrefixCache:
    """Automatic prefix caching — the vLLM ``--enable-prefix-caching`` / LMCache chunk-reuse role
    (``LLM_on_Kubernetes/Inference_Platfrom/07-L1-Cache``, README "APC": system-prompt /
    RAG-document / multi-turn TTFT reductions).

    Prompts are cut into ``block``-token chunks identified by a chained content hash (blake2b of
    the previous chunk's digest + this chunk's token ids — stable across processes, so TP ranks
    and restarts agree without PYTHONHASHSEED).  Each cached chunk keeps its K/V rows for every
    layer in an HBM pool ``[layers][capacity, block, Hkv·D]``; a hit copies the longest cached
    chunk run into the request's KV slot (one gather per layer) and only the suffix is
    prefilled.  LRU eviction; at least one prompt token is always recomputed (its logits seed
    the first sampled token).

    Host tier (LMCache ``LMCACHE_LOCAL_CPU`` / ``max_local_cpu_size`` role,
    ``07-L1-Cache/LMCache/vllm-statefulset-lmcache.yaml:96-111``): with ``host_blocks > 0`` a chunk
    evicted from HBM is spilled to a pinned host pool instead of dropped, and a later hit restores
    it over PCIe into a free HBM block (its own LRU; the HBM pool holds the hot set, host memory
    — hundreds of GB on an MI355X node — the warm set).

    Remote tier (LMCache server role, ``07-L1-Cache/LMCache/lmcache-deployment.yaml``): with a
    :class:`~.kv_server.RemoteKV`, every newly computed chunk is written through to a store shared
    by all replicas (write-behind, off the engine loop), and a chunk missing from HBM and host is
    fetched from it before giving up — a prefix prefilled on one replica is warm on all of them.

    ``namespace`` seeds every chain: the engine derives it from the model identity (name, a
    fingerprint of the weights, dtype, layer count, KV width, block size, TP rank), so two
    deployments sharing one remote store (a base and a fine-tuned model of the same shape) never
    read each other's K/V — LMCache's keys carry the model name and format for the same reason.
    ``salt`` separates hash chains whose K/V differ for the same tokens (multi-LoRA adapters); the
    engine passes the adapter's NAME and path, not its slot index (which depends on the order of
    ``--lora-modules``)."""

    def __init__(self, n_layers: int, width: int, dtype, device, block: int = 64, capacity_blocks: int = 512,
                 host_blocks: int = 0, remote=None, namespace: bytes = b""):
        import collections
        self.namespace = bytes(namespace)
        self.remote = remote
        self.remote_hits = 0
        self.block, self.capacity = block, capacity_blocks
        self.k = [torch.zeros(capacity_blocks, block, width, dtype=dtype, device=device) for _ in range(n_layers)]
        self.v = [torch.zeros(capacity_blocks, block, width, dtype=dtype, device=device) for _ in range(n_layers)]
        self.map: "collections.OrderedDict[bytes, int]" = collections.OrderedDict()
        self.free = list(range(capacity_blocks))
        self.hit_tokens = 0
        self.query_tokens = 0
        self.host_blocks = int(host_blocks)
        self.host_hits = 0
        self.spills = 0
        if self.host_blocks > 0:
            pin = torch.device(device).type == "cuda"
            shape = (n_layers, 2, self.host_blocks, block, width)
            self.host = torch.zeros(shape, dtype=dtype, pin_memory=pin)
            self.hmap: "collections.OrderedDict[bytes, int]" = collections.OrderedDict()
            self.hfree = list(range(self.host_blocks))

    def _digests(self, ids: list[int], n_blocks: int, salt: bytes | int = 0) -> list[bytes]:
        import hashlib
        if isinstance(salt, int):
            salt = b"" if not salt else salt.to_bytes(8, "little")
        prev = self.namespace + (b"|" + salt if salt else b"")
        if prev:
            prev = hashlib.blake2b(prev, digest_size=16).digest()
        out = []
        for i in range(n_blocks):
            h = hashlib.blake2b(prev, digest_size=16)
            h.update(torch.tensor(ids[i * self.block:(i + 1) * self.block], dtype=torch.int32).numpy().tobytes())
            prev = h.digest()
            out.append(prev)
        return out

    # ---- host tier ---------------------------------------------------------------------
    def _alloc_hbm(self) -> int:
        """A free HBM block; the LRU one is spilled to the host tier (or dropped) first."""
        if not self.free:
            d, j = self.map.popitem(last=False)
            if self.host_blocks > 0 and d not in self.hmap:
                if not self.hfree:
                    _, hj = self.hmap.popitem(last=False)
                    self.hfree.append(hj)
                hj = self.hfree.pop()
                for l in range(len(self.k)):
                    self.host[l, 0, hj].copy_(self.k[l][j], non_blocking=True)
                    self.host[l, 1, hj].copy_(self.v[l][j], non_blocking=True)
                self.hmap[d] = hj
                self.spills += 1
            self.free.append(j)
        return self.free.pop()

    def _restore(self, d: bytes) -> int | None:
        hj = self.hmap.get(d) if self.host_blocks > 0 else None
        if hj is None:
            return None
        if self.k[0].is_cuda:
            torch.cuda.current_stream().synchronize()     # spills of the same step have landed
        j = self._alloc_hbm()
        for l in range(len(self.k)):
            self.k[l][j].copy_(self.host[l, 0, hj], non_blocking=True)
            self.v[l][j].copy_(self.host[l, 1, hj], non_blocking=True)
        self.hmap.move_to_end(d)
        self.map[d] = j
        self.host_hits += 1
        return j

    # ---- remote tier ---------------------------------------------------------------------
    def _chunk_shape(self):
        return (len(self.k), 2, self.block, self.k[0].shape[-1])

    def _remote_fetch(self, d: bytes) -> int | None:
        if self.remote is None:
            return None
        data = self.remote.get(d)
        L, _, B, W = self._chunk_shape()
        esz = self.k[0].element_size()
        if data is None or len(data) != L * 2 * B * W * esz:
            return None
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).view(self.k[0].dtype).view(L, 2, B, W)
        if self.k[0].is_cuda:
            t = t.pin_memory()
        j = self._alloc_hbm()
        for l in range(L):
            self.k[l][j].copy_(t[l, 0], non_blocking=True)
            self.v[l][j].copy_(t[l, 1], non_blocking=True)
        if self.k[0].is_cuda:
            torch.cuda.current_stream().synchronize()     # the pinned staging buffer dies here
        self.map[d] = j
        self.remote_hits += 1
        return j

    def _remote_write(self, digests: list[bytes], dst: "torch.Tensor"):
        """Write-through of freshly stored chunks: one D2H gather into pinned memory on the current
        stream, bytes produced and uploaded on the client's writer thread after the copy lands."""
        L = len(self.k)
        stacked = torch.stack([torch.stack([self.k[l][dst], self.v[l][dst]]) for l in range(L)])   # [L,2,n,B,W]
        if stacked.is_cuda:
            host = torch.empty(stacked.shape, dtype=stacked.dtype, pin_memory=True)
            host.copy_(stacked, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = stacked.clone(), None
        for i, d in enumerate(digests):
            def payload(i=i):
                if ev is not None:
                    ev.synchronize()
                return host[:, :, i].contiguous().view(torch.uint8).numpy().tobytes()
            self.remote.put(d, payload)

    def match(self, ids: list[int], salt: bytes | int = 0) -> list[int]:
        """Pool indices of the longest cached chunk run (leaving >= 1 token to prefill)."""
        n = (len(ids) - 1) // self.block
        idx = []
        for d in self._digests(ids, n, salt):
            j = self.map.get(d)
            if j is None:
                j = self._restore(d)
                if j is None:
                    j = self._remote_fetch(d)
                if j is None:
                    break
            self.map.move_to_end(d)
            idx.append(j)
        self.query_tokens += len(ids)
        self.hit_tokens += len(idx) * self.block
        return idx

    def load(self, idx: list[int], cache: KVCache, slot: int):
        n = len(idx) * self.block
        t = torch.tensor(idx, device=self.k[0].device)
        for l in range(len(self.k)):
            cache.k[l][slot, :n] = self.k[l][t].reshape(n, -1)
            cache.v[l][slot, :n] = self.v[l][t].reshape(n, -1)

    def store(self, ids: list[int], cache: KVCache, slot: int, salt: bytes | int = 0):
        """Insert every full prompt chunk of a freshly prefilled slot that is not cached yet."""
        n = len(ids) // self.block
        new = []
        digests = self._digests(ids, n, salt)
        for i, d in enumerate(digests):
            if d in self.map:
                self.map.move_to_end(d)
                continue
            j = self._alloc_hbm()                            # evicts (spills) the LRU block if full
            self.map[d] = j
            new.append((i, j))
        if not new:
            return
        src = torch.tensor([i for i, _ in new], device=self.k[0].device)
        dst = torch.tensor([j for _, j in new], device=self.k[0].device)
        B = self.block
        for l in range(len(self.k)):
            self.k[l][dst] = cache.k[l][slot, :n * B].view(n, B, -1)[src]
            self.v[l][dst] = cache.v[l][slot, :n * B].view(n, B, -1)[src]
        if self.remote is not None:
            self._remote_write([digests[i] for i, _ in new], dst)


@dataclasses.dataclass
class _Slot:
    req: _Request
    gen: list = dataclasses.field(default_factory=list)
    sent: int = 0
    text: str = ""                       # streamed/stop-checked text so far (incremental detokenisation)
    poff: int = 0                        # gen[poff:roff] = context tokens of the last emitted piece
    roff: int = 0
    t_first: float | None = None
    prefilled: int = -1                  # chunked prefill: prompt tokens in the cache so far (-1 = decoding)
    done: bool = False
    finish: str = "length"


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


def _unwrap_lm(model):
    m = model
    for _ in range(4):
        bm = getattr(m, "__dict__", {}).get("_modules", {}).get("base_model")
        if bm is not None and hasattr(bm, "model"):      # PeftModel: unwrap before duck-typing
            m = bm.model
            continue
        if hasattr(m, "lm_head") and hasattr(m, "model"):
            return m
        m = getattr(m, "model", None) or getattr(m, "module", None)
        if m is None:
            break
    raise TypeError("ServingEngine needs a causal LM with .model and .lm_head")


def kv_slots_for_budget(total_bytes: int, used_bytes: int, fraction: float, slot_bytes: int,
                        reserve_bytes: int = 0) -> int:
    """vLLM ``--gpu-memory-utilization`` semantics: the engine may occupy ``fraction`` of the device's memory;
    what the resident weights (``used_bytes``) and the prefill activation reserve leave of it holds the KV
    cache — here whole sequence slots of ``max_model_len`` tokens (the contiguous cache below).  Raises, like
    vLLM, when not even one slot fits."""
    if not 0.0 < fraction <= 1.0:
        raise ValueError(f"gpu_memory_utilization {fraction}: must be in (0, 1]")
    budget = fraction * total_bytes - used_bytes - reserve_bytes
    if budget < slot_bytes:
        raise ValueError(f"no memory for the KV cache at gpu_memory_utilization={fraction}: "
                         f"{budget / 2 ** 30:.2f} GiB left after weights and activations, one "
                         f"{slot_bytes / 2 ** 30:.2f} GiB sequence slot needed (raise the fraction or lower "
                         f"--max-model-len)")
    return int(budget // slot_bytes)


class ServingEngine:
    def __init__(self, model, tokenizer, model_name: str = "lipa-model", max_batch: int = 16,
                 system_prompt: str | None = None, chat_template: str = "auto", space_before_end: bool = False,
                 max_model_len: int | None = None, max_prefill_batch: int | None = None, prefill_token_budget: int = 16384,
                 use_graphs: bool | None = None, tp_group=None, prefix_cache_blocks: int = 0,
                 prefix_block: int = 64, chunked_prefill: int = 0, lora_modules: dict[str, str] | None = None,
                 host_cache_blocks: int = 0, kv_remote_url: str | None = None,
                 gpu_memory_utilization: float | None = None):
        """``tp_group``: the model was sharded by ``parallel.tensor_parallel`` over this group.
        The engine then runs SPMD — group rank 0 owns the request queue and broadcasts each
        iteration's admissions; the other ranks call :meth:`follower_loop` and replay exactly the
        same prefill / decode / sampling (logits are bit-identical across ranks, the samplers
        are seeded identically), so no tokens need to be exchanged."""
        self.model, self.tok, self.model_name = model, tokenizer, model_name
        # vLLM --enable-chunked-prefill: prompts longer than this many tokens are prefilled one
        # chunk per engine iteration, interleaved with the running batch's decode steps
        self.chunked_prefill = int(chunked_prefill or 0)
        self.tp_group = tp_group
        self.tp_rank = 0
        if tp_group is not None:
            import torch.distributed as dist
            self.tp_rank = dist.get_rank(tp_group)
            self.tp_src = dist.get_global_rank(tp_group, 0) if hasattr(dist, "get_global_rank") else 0
            use_graphs = False                 # collectives stay eager (no capture of RCCL calls)
            from ..ops.decode import seed_sampler
            seed_sampler(1234)
            torch.manual_seed(1234)
        self.lm = _unwrap_lm(model)
        self.lm.eval()
        self.max_batch = max_batch
        # admit a whole burst at once (one packed prefill, bounded by the token budget) rather than in
        # waves of 32: every wave costs the waiting requests another prefill + decode iteration
        self.max_prefill_batch = max_prefill_batch or max_batch
        self.prefill_token_budget = prefill_token_budget
        self.system_prompt = system_prompt
        self.chat_template = chat_template
        self.space_before_end = space_before_end
        self.device = next(model.parameters()).device
        cfg = self.lm.config
        self.max_len = int(max_model_len or min(getattr(cfg, "max_position_embeddings", 4096), 4096))
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
                      "batches_total": 0, "running": 0, "decode_steps_total": 0}
        self.h_latency = _Histogram([0.05, 0.1, 0.25, 0.5, 1, 2, 5, 10, 30, 60])
        self.h_ttft = _Histogram([0.01, 0.025, 0.05, 0.1, 0.2, 0.5, 1, 2, 5])
        self.queue_time_ewma: float | None = None
        if gpu_memory_utilization is not None and self.device.type == "cuda":
            # the KV pool sized from the memory fraction (vLLM --gpu-memory-utilization), capped by max_batch
            elt = torch.finfo(self.lm.lm_head.weight.dtype).bits // 8
            slot = 2 * cfg.num_hidden_layers * self.max_len * cfg.num_key_value_heads * cfg.head_dim * elt
            reserve = (2 << 30) + prefill_token_budget * (16 * cfg.hidden_size + 6 * getattr(cfg, "intermediate_size", 0))
            fit = kv_slots_for_budget(torch.cuda.get_device_properties(self.device).total_memory,
                                      torch.cuda.memory_allocated(self.device), gpu_memory_utilization, slot, reserve)
            max_batch = max(1, min(max_batch, fit))
            self.max_batch = max_batch
            self.max_prefill_batch = min(self.max_prefill_batch, max_batch)
        self.cache = KVCache(cfg.num_hidden_layers, max_batch, self.max_len, cfg.num_key_value_heads, cfg.head_dim,
                             self.lm.lm_head.weight.dtype, self.device)
        self.cache.pos = torch.zeros(max_batch, dtype=torch.long, device=self.device)
        self.prefix = None
        remote = None
        if kv_remote_url and prefix_cache_blocks > 0:
            from .kv_server import RemoteKV
            remote = RemoteKV(kv_remote_url)
        if prefix_cache_blocks > 0:
            self.prefix = PrefixCache(cfg.num_hidden_layers, cfg.num_key_value_heads * cfg.head_dim,
                                      self.lm.lm_head.weight.dtype, self.device, prefix_block, prefix_cache_blocks,
                                      host_blocks=host_cache_blocks, remote=remote,
                                      namespace=self._kv_namespace(prefix_block))
        # multi-LoRA serving (vLLM --enable-lora --lora-modules): stacked adapters, per-row masks;
        # built BEFORE the decode graphs are captured so the adapter term is part of every graph
        self.mlora = None
        if lora_modules:
            from ..peft.multi_lora import MultiLoraManager
            self.mlora = MultiLoraManager(self.lm, dict(lora_modules), max_rows=max_batch)
        # prefix-cache chain salt per adapter slot: its name and path (slot 0 = the base model)
        self._adapter_salt = [b""] + [f"{n}={p}".encode() for n, p in (lora_modules or {}).items()]
        if self.mlora is not None:
            self._adapter_salt = [b""] * (1 + len(self.mlora.names))
            for n, i in self.mlora.index.items():
                self._adapter_salt[i] = f"{n}={(lora_modules or {}).get(n, '')}".encode()
        self.slots: list[_Slot | None] = [None] * max_batch
        self.next_tok = torch.full((max_batch,), self.pad, dtype=torch.long, device=self.device)
        self.graphs = None
        if use_graphs is None:
            use_graphs = self.device.type == "cuda"
        if use_graphs:                     # one hipGraph per batch bucket (infer/graphs.py)
            from .graphs import DecodeGraphs
            with torch.no_grad():
                self.graphs = DecodeGraphs(self.lm, self.cache, max_batch, tokens=self.next_tok)
        self._held: _Request | None = None
        self._admitting = None
        self.iteration_hook = None               # engine-process mode: flush the batched outputs
        self._pending = None                     # (pinned host tokens, event, owners) of the in-flight step
        self.pipeline = self.device.type == "cuda"
        self._stop = False
        self._closing = False
        self._worker = None
        if self.tp_rank == 0:
            self._worker = threading.Thread(target=self._loop, daemon=True)
            self._worker.start()

    def follower_loop(self):
        """TP ranks > 0: replay rank 0's iterations until it shuts down."""
        self._loop()

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

    def _kv_namespace(self, block: int) -> bytes:
        """Model identity for the prefix-cache keys: served name, dims, dtype, block size, TP rank and
        a fingerprint of the weights (a few rows of the embedding, the head and the last layer's
        parameters — enough to tell a base model from its fine-tune of the same architecture)."""
        import hashlib
        cfg = self.lm.config
        h = hashlib.blake2b(digest_size=16)
        h.update(f"{self.model_name}|{cfg.num_hidden_layers}|{cfg.num_key_value_heads}|{cfg.head_dim}|"
                 f"{self.lm.lm_head.weight.dtype}|{block}|tp{self.tp_rank}".encode())
        params = list(self.lm.parameters())
        with torch.no_grad():
            for p in (params[0], params[-1], self.lm.lm_head.weight):
                t = p.detach().reshape(-1)[:4096].float().cpu()
                h.update(t.numpy().tobytes())
        return h.digest()

    def _salt(self, adapter: int) -> bytes:
        return self._adapter_salt[adapter] if 0 <= adapter < len(self._adapter_salt) else str(adapter).encode()

    # ------------------------------------------------------------------ request API (thread-safe)
    @property
    def served_models(self) -> list[str]:
        """``/v1/models``: the base model plus every LoRA adapter name."""
        return [self.model_name] + (list(self.mlora.names) if self.mlora is not None else [])

    def adapter_id(self, model: str | None) -> int:
        """Request ``model`` → adapter index; KeyError for a model this server does not serve."""
        if model is None or model == self.model_name:
            return 0
        if self.mlora is None or model not in self.mlora.index:
            raise KeyError(model)
        return self.mlora.index[model]

    def submit(self, prompt: str, params: SamplingParams, stream: bool = False, model: str | None = None,
               out=None) -> _Request:
        """``out``: any object with a thread-safe ``put`` (default a ``queue.Queue``); the HTTP server
        passes an :class:`AsyncOut` so streamed deltas reach its event loop without a thread hop
        per token."""
        room = self.max_len - 1 - min(params.max_tokens, self.max_len // 2)   # keep space to generate
        ids = self.encode(prompt)[-room:]
        r = _Request(ids, params, stream, out if out is not None else queue.Queue(), time.time(),
                     adapter=self.adapter_id(model))
        self.q.put(r)
        return r

    def complete(self, prompt: str, params: SamplingParams, timeout: float | None = None,
                 model: str | None = None) -> dict:
        r = self.submit(prompt, params, stream=False, model=model)
        while True:
            kind, val = r.out.get(timeout=timeout)
            if kind == "final":
                return val
            if kind == "error":
                raise RuntimeError(val)

    def stream(self, prompt: str, params: SamplingParams, timeout: float | None = None, model: str | None = None):
        r = self.submit(prompt, params, stream=True, model=model)
        while True:
            kind, val = r.out.get(timeout=timeout)
            if kind == "delta":
                yield val, None
            elif kind == "final":
                yield "", val
                return
            elif kind == "error":
                raise RuntimeError(val)

    def shutdown(self, timeout: float = 30.0):
        """Stop the engine loop and wait for it, so no GPU work is in flight while the caller (or
        the interpreter) tears down graphs and allocators."""
        if self.tp_group is None:
            self._stop = True
        else:   # SPMD: rank 0 must hand the stop to its followers inside the iteration protocol
            self._closing = True
        self.q.put(None)
        w = self._worker
        if w is not None and w is not threading.current_thread():
            w.join(timeout)

    # ------------------------------------------------------------------ worker
    def _loop(self):
        while not self._stop:
            try:
                self._iteration()
                if self.iteration_hook is not None:
                    self.iteration_hook()
            except Exception as e:  # fail the in-flight requests (incl. ones being admitted), keep serving
                self._pending = None
                failed = set()
                for i, s in enumerate(self.slots):
                    if s is not None:
                        s.req.out.put(("error", repr(e)))
                        failed.add(id(s.req))
                        self.slots[i] = None
                for _, r in (self._admitting or []):
                    if id(r) not in failed:
                        r.out.put(("error", repr(e)))
                self._admitting = None
                self.cache.pos.zero_()
                if self.iteration_hook is not None:
                    self.iteration_hook()

    def _iteration(self):
        new = self._collect() if self.tp_rank == 0 else []
        if self._closing and self.tp_rank == 0:
            new = None
        if self.tp_group is not None:
            new = self._tp_sync(new)
        if new is None:
            self._stop = True
            return
        with self.lock, torch.no_grad():
            if new:
                self._admitting = new
                self._admit(new)
                self._admitting = None
            if self.chunked_prefill:
                self._prefill_chunks()
            if any(s is not None and s.prefilled < 0 for s in self.slots):
                self._decode_step()
            else:
                self._flush_pending()            # only finished requests' extra tokens can be in flight

    def _tp_sync(self, new):
        """Broadcast this iteration's admissions (slot, prompt ids, sampling params) from TP rank 0."""
        import torch.distributed as dist
        payload = None if new is None else [(slot, r.prompt_ids, dataclasses.asdict(r.params), r.t_arrive, r.adapter)
                                            for slot, r in new]
        box = [payload]
        dist.broadcast_object_list(box, src=self.tp_src, group=self.tp_group)
        if self.tp_rank == 0:
            return new
        if box[0] is None:
            return None
        return [(slot, _Request(ids, SamplingParams(**pd), False, queue.Queue(), t, adapter=a))
                for slot, ids, pd, t, a in box[0]]

    def _collect(self):
        """Pull the requests to admit this iteration (None = shut down)."""
        active = [i for i, s in enumerate(self.slots) if s is not None]
        free = [i for i, s in enumerate(self.slots) if s is None]
        new = []
        block = not active
        budget = self.prefill_token_budget
        while free and len(new) < self.max_prefill_batch:
            if self._held is not None:
                r, self._held = self._held, None
            else:
                try:
                    # idle TP ranks wait inside a collective: heartbeat once a second
                    tmo = (1.0 if self.tp_group is not None else None) if block else 0
                    r = self.q.get(block=block, timeout=tmo)
                except queue.Empty:
                    break
            block = False
            if r is None:
                return None
            if new and len(r.prompt_ids) > budget:      # over the prefill token budget: next iteration
                self._held = r
                break
            budget -= len(r.prompt_ids)
            qt = max(0.0, time.time() - r.t_arrive)     # router load signal (llm-d queue_time_ms)
            self.queue_time_ewma = qt if self.queue_time_ewma is None else 0.8 * self.queue_time_ewma + 0.2 * qt
            new.append((free.pop(0), r))
        return new

    def _admit(self, new):
        """Prefill the new prompts together into a scratch cache, copy into their slots, sample
        each one's first token.  With prefix caching, prompts whose leading chunks are cached
        load them and prefill only their suffix (one request at a time).  With chunked prefill,
        prompts longer than the chunk are only registered here (see :meth:`_prefill_chunks`)."""
        if self.mlora is not None:
            for slot, r in new:
                self.mlora.set_slot(slot, r.adapter)
        if self.chunked_prefill:
            short = []
            for slot, r in new:
                if len(r.prompt_ids) > self.chunked_prefill:
                    P = 0
                    if self.prefix is not None:
                        idx = self.prefix.match(r.prompt_ids, self._salt(r.adapter))
                        if idx:
                            self.prefix.load(idx, self.cache, slot)
                            P = len(idx) * self.prefix.block
                    self.slots[slot] = _Slot(r, prefilled=P)
                    self.cache.pos[slot] = P
                else:
                    short.append((slot, r))
            new = short
            if not new:
                return
        if self.prefix is not None:
            rest = []
            for slot, r in new:
                idx = self.prefix.match(r.prompt_ids, self._salt(r.adapter))
                if idx:
                    self._admit_suffix(slot, r, idx)
                else:
                    rest.append((slot, r))
            if rest:
                self._admit_batch(rest)
            for slot, r in new:      # (a slot that already finished keeps its rows until reused)
                self.prefix.store(r.prompt_ids, self.cache, slot, self._salt(r.adapter))
            return
        self._admit_batch(new)

    def _rows_for(self, parts: list[tuple[int, int]]):
        """Multi-LoRA: install the per-token adapter index of a prefill batch [(adapter, n_tokens)]."""
        if self.mlora is not None:
            self.mlora.use_rows(torch.cat([torch.full((n,), a, dtype=torch.long) for a, n in parts]).to(self.device))

    def _rows_done(self):
        if self.mlora is not None:
            self.mlora.use_rows(None)

    def _slot_view(self, slot: int, length: int) -> KVCache:
        view = KVCache.__new__(KVCache)
        view.k = [t[slot:slot + 1] for t in self.cache.k]
        view.v = [t[slot:slot + 1] for t in self.cache.v]
        view.len, view.max_len, view.batch, view.pos = length, self.cache.max_len, 1, None
        view._rows = self.cache._rows[:1]
        return view

    def _prefill_chunks(self):
        """One chunk of at most ``chunked_prefill`` prompt tokens (oldest prefilling slot first)
        per iteration; the chunk attends to the slot's cached prefix.  The last chunk samples the
        request's first token and the slot joins the decode batch."""
        pre = sorted((i for i, s in enumerate(self.slots) if s is not None and s.prefilled >= 0),
                     key=lambda i: self.slots[i].req.t_arrive)
        if not pre:
            return
        slot = pre[0]
        s = self.slots[slot]
        r, P = s.req, s.prefilled
        L = len(r.prompt_ids)
        C = min(self.chunked_prefill, L - P)
        ids = torch.tensor([r.prompt_ids[P:P + C]], dtype=torch.long, device=self.device)
        self._rows_for([(r.adapter, C)])
        try:
            h = self.lm.model(ids, None, self._slot_view(slot, P), None)
        finally:
            self._rows_done()
        s.prefilled = P + C
        self.cache.pos[slot] = P + C
        self.stats["batches_total"] += 1
        if P + C < L:
            return
        s.prefilled = -1
        self.stats["prompt_tokens_total"] += L
        logits = head_logits(h[-1:], self.lm.lm_head.weight)
        dev_toks, toks = self._sample(logits, [slot])
        self.next_tok[slot] = dev_toks[0]
        if self.prefix is not None:
            self.prefix.store(r.prompt_ids, self.cache, slot, self._salt(r.adapter))
        self._accept(slot, toks[0], time.time())

    def _admit_suffix(self, slot, r, idx):
        lm = self.lm
        P = len(idx) * self.prefix.block
        self.prefix.load(idx, self.cache, slot)
        view = self._slot_view(slot, P)
        ids = torch.tensor([r.prompt_ids[P:]], dtype=torch.long, device=self.device)
        self._rows_for([(r.adapter, len(r.prompt_ids) - P)])
        try:
            h = lm.model(ids, None, view, None)
        finally:
            self._rows_done()
        logits = head_logits(h[-1:], lm.lm_head.weight)
        L = len(r.prompt_ids)
        self.cache.pos[slot] = L
        self.slots[slot] = _Slot(r)
        self.stats["prompt_tokens_total"] += L
        dev_toks, toks = self._sample(logits, [slot])
        self.next_tok[slot] = dev_toks[0]
        self._accept(slot, toks[0], time.time())
        self.stats["batches_total"] += 1

    def _admit_batch(self, new):
        """Prefill the admitted prompts packed back to back (no padding) directly into their
        cache slots (models/common.py ``PackedPrefill``), sample each one's first token."""
        lm = self.lm
        lens = [len(r.prompt_ids) for _, r in new]
        ids = torch.tensor([[t for _, r in new for t in r.prompt_ids]], dtype=torch.long).to(self.device)
        pp = PackedPrefill(self.cache, [s for s, _ in new], lens, self.device)
        self._rows_for([(r.adapter, n) for (_, r), n in zip(new, lens)])
        try:
            h = lm.model(ids, pp.positions, pp, None)
        finally:
            self._rows_done()
        logits = head_logits(h[pp.last], lm.lm_head.weight)
        rows = torch.tensor([s for s, _ in new], device=self.device)
        self.cache.pos[rows] = torch.tensor(lens, dtype=torch.long, device=self.device)
        now = time.time()
        for b, (slot, r) in enumerate(new):
            self.slots[slot] = _Slot(r)
            self.stats["prompt_tokens_total"] += len(r.prompt_ids)
        dev_toks, toks = self._sample(logits, [s for s, _ in new])
        self.next_tok[rows] = dev_toks
        for b, (slot, r) in enumerate(new):
            self._accept(slot, toks[b], now)
        self.stats["batches_total"] += 1

    def _sample(self, logits, slot_ids):
        """Sample one token per row, grouping rows with identical sampling parameters.
        Returns (device tensor, host list)."""
        out = self._sample_dev(logits, slot_ids)
        return out, out.tolist()

    def _sample_dev(self, logits, slot_ids):
        out = torch.empty(len(slot_ids), dtype=torch.long, device=self.device)
        groups: dict = {}
        for j, s in enumerate(slot_ids):
            groups.setdefault(self.slots[s].req.params.key(), []).append(j)
        for (temp, top_p, top_k, pen), js in groups.items():
            idx = None if len(groups) == 1 else torch.tensor(js, device=self.device)
            hist = None
            if pen != 1.0:
                L = max(len(self.slots[slot_ids[j]].req.prompt_ids) + len(self.slots[slot_ids[j]].gen) for j in js)
                hist = torch.full((len(js), max(1, L)), -1, dtype=torch.int32)
                for q, j in enumerate(js):
                    s = self.slots[slot_ids[j]]
                    seq = s.req.prompt_ids + s.gen
                    hist[q, :len(seq)] = torch.tensor(seq, dtype=torch.int32)
                hist = hist.to(self.device)
            if idx is None:
                out = sample(logits.float(), hist, temp, top_k, top_p, pen)
            else:
                out[idx] = sample(logits[idx].float(), hist, temp, top_k, top_p, pen)
        return out

    def _accept(self, slot: int, tok: int, now: float):
        s = self.slots[slot]
        if s.t_first is None:
            s.t_first = now
        p = s.req.params
        if tok in self.eos and not p.ignore_eos:
            s.done, s.finish = True, "stop"
        else:
            s.gen.append(tok)
            if len(s.gen) >= p.max_tokens or len(s.req.prompt_ids) + len(s.gen) >= self.max_len - 1:
                s.done, s.finish = True, "length"
            if s.req.stream or p.stop:
                # incremental detokenisation: decode only the few tokens since the last emitted
                # piece (plus their left context), not the whole generation every step
                prev = self.tok.decode(s.gen[s.poff:s.roff], skip_special_tokens=True)
                cur = self.tok.decode(s.gen[s.poff:], skip_special_tokens=True)
                if len(cur) > len(prev) and not cur.endswith("\ufffd"):
                    new = cur[len(prev):]
                    s.poff, s.roff = s.roff, len(s.gen)
                    s.text += new
                    if s.req.stream:
                        s.req.out.put(("delta", new))
                        s.sent = len(s.text)
                    if p.stop:
                        tail = s.text[-(len(new) + max(len(st) for st in p.stop)):]
                        if any(st and st in tail for st in p.stop):
                            s.done, s.finish = True, "stop"
        if s.done:
            self._finish(slot)

    def _finish(self, slot: int):
        s = self.slots[slot]
        r = s.req
        text = self.tok.decode(s.gen, skip_special_tokens=True)
        if r.params.stop:
            cut = min((text.find(st) for st in r.params.stop if st and st in text), default=-1)
            if cut >= 0:
                text = text[:cut]
        if r.stream and len(text) > len(s.text) and text.startswith(s.text):
            r.out.put(("delta", text[len(s.text):]))       # flush a held-back partial character
        t1 = time.time()
        self.stats["requests_total"] += 1
        self.stats["generation_tokens_total"] += len(s.gen)
        self.h_latency.observe(t1 - r.t_arrive)
        if s.t_first is not None:
            self.h_ttft.observe(s.t_first - r.t_arrive)
        r.out.put(("final", {"text": text, "finish_reason": s.finish, "prompt_tokens": len(r.prompt_ids),
                             "completion_tokens": len(s.gen), "latency_s": t1 - r.t_arrive,
                             "ttft_s": (s.t_first or t1) - r.t_arrive}))
        self.slots[slot] = None
        self.cache.pos[slot] = 0

    def _decode_step(self):
        lm = self.lm
        active = [i for i, s in enumerate(self.slots) if s is not None and s.prefilled < 0]
        self.stats["running"] = len(active)
        n = active[-1] + 1                       # slots fill lowest-first: decode rows [0, n) only
        if self.graphs is not None:              # hipGraph replay of the whole step (bucket >= n rows)
            n = self.graphs.bucket(n)
            logits = self.graphs.step(None, n)
        else:
            h = lm.model(self.next_tok[:n, None], None, self.cache.head_rows(n), None)   # per-row positions
            logits = head_logits(h, lm.lm_head.weight)
        free = [i for i in range(n) if self.slots[i] is None]
        if free:                                                              # idle rows stay at position 0
            self.cache.pos[torch.tensor(free, device=self.device)] = 0
        for i in range(n):       # a slot mid chunked-prefill decoded a junk row at its next prompt position
            s = self.slots[i]     # (the next chunk overwrites it): put its position back
            if s is not None and s.prefilled >= 0:
                self.cache.pos[i] = s.prefilled
        rows = torch.tensor(active, device=self.device)
        if len(active) != n:
            logits = logits[rows]
        if self.pipeline and all(self.slots[s].req.params.repetition_penalty == 1.0 for s in active):
            # asynchronous: the sampled tokens stay on the device (next step's input), a pinned
            # copy + event hand them to the host, and the host accepts the PREVIOUS step's
            # tokens while this step runs on the GPU (a finished request decodes one extra,
            # discarded token)
            dev_toks = self._sample_dev(logits, active)
            self.next_tok[rows] = dev_toks
            host = torch.empty(len(active), dtype=torch.long, pin_memory=True)
            host.copy_(dev_toks, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            prev, self._pending = self._pending, (host, ev, [(sl, self.slots[sl].req) for sl in active])
            if prev is not None:
                self._process_pending(prev)
        else:
            self._flush_pending()
            dev_toks, toks = self._sample(logits, active)
            self.next_tok[rows] = dev_toks
            now = time.time()
            for j, slot in enumerate(active):
                self._accept(slot, toks[j], now)
        self.stats["decode_steps_total"] += 1
        self.stats["running"] = sum(s is not None for s in self.slots)

    def _process_pending(self, pend):
        host, ev, owners = pend
        ev.synchronize()
        now = time.time()
        for (slot, req), tok in zip(owners, host.tolist()):
            s = self.slots[slot]
            if s is not None and s.req is req and not s.done:
                self._accept(slot, tok, now)

    def _flush_pending(self):
        if self._pending is not None:
            p, self._pending = self._pending, None
            self._process_pending(p)

    # ------------------------------------------------------------------ metrics
    def prometheus(self) -> str:
        s = self.stats
        lines = [
            "# TYPE lipa_requests_total counter", f"lipa_requests_total {s['requests_total']}",
            "# TYPE lipa_prompt_tokens_total counter", f"lipa_prompt_tokens_total {s['prompt_tokens_total']}",
            "# TYPE lipa_generation_tokens_total counter",
            f"lipa_generation_tokens_total {s['generation_tokens_total']}",
            "# TYPE lipa_decode_steps_total counter", f"lipa_decode_steps_total {s['decode_steps_total']}",
            "# TYPE lipa_batches_total counter", f"lipa_batches_total {s['batches_total']}",
            "# TYPE lipa_num_requests_waiting gauge", f"lipa_num_requests_waiting {self.q.qsize()}",
            "# TYPE lipa_num_requests_running gauge", f"lipa_num_requests_running {s['running']}",
        ]
        # KV occupancy: rows held by live slots over the cache capacity (vLLM gpu_cache_usage_perc role)
        used = 0
        try:
            pos = self.cache.pos.tolist() if self.cache.pos is not None else []
            used = sum(int(pos[i]) for i, sl in enumerate(self.slots) if sl is not None and i < len(pos))
        except Exception:
            pass
        cap = max(1, self.max_batch * self.cache.max_len)
        lines += ["# TYPE lipa_gpu_cache_usage_perc gauge", f"lipa_gpu_cache_usage_perc {used / cap:.6f}",
                  "# TYPE lipa_queue_time_seconds gauge", f"lipa_queue_time_seconds {self.queue_time_ewma or 0.0:.6f}"]
        if self.prefix is not None:
            lines += ["# TYPE lipa_prefix_cache_queries_total counter",
                      f"lipa_prefix_cache_queries_total {self.prefix.query_tokens}",
                      "# TYPE lipa_prefix_cache_hits_total counter",
                      f"lipa_prefix_cache_hits_total {self.prefix.hit_tokens}",
                      "# TYPE lipa_prefix_cache_host_hits_total counter",
                      f"lipa_prefix_cache_host_hits_total {self.prefix.host_hits}",
                      "# TYPE lipa_prefix_cache_spills_total counter",
                      f"lipa_prefix_cache_spills_total {self.prefix.spills}",
                      "# TYPE lipa_prefix_cache_remote_hits_total counter",
                      f"lipa_prefix_cache_remote_hits_total {self.prefix.remote_hits}"]
        lines += self.h_latency.render("lipa_e2e_request_latency_seconds")
        lines += self.h_ttft.render("lipa_time_to_first_token_seconds")
        if torch.cuda.is_available():
            lines += ["# TYPE lipa_hbm_allocated_bytes gauge",
                      f"lipa_hbm_allocated_bytes {torch.cuda.memory_allocated()}"]
        return "\n".join(lines) + "\n"
