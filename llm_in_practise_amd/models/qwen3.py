"""Native Qwen3 causal LM (Qwen3-4B/8B/14B, DeepSeek-R1-0528-Qwen3-8B).

Replaces the reference's ``AutoModelForCausalLM.from_pretrained(<Qwen3 dir>)``
(``Fine-Tuning/qwen3-8b-qlora.py:86-101``, ``deepseek-r1-0528-qwen3-8b-qlora.dist.py:99-112``).
Module names match HF's ``Qwen3ForCausalLM`` so safetensors checkpoints load as-is and
PEFT adapter keys (``base_model.model.model.layers.{i}.self_attn.q_proj.lora_A.weight``)
line up.  Architecture [ext: public HF config]: RMSNorm (eps 1e-6), GQA attention with
per-head q/k RMSNorm, rotate-half RoPE (θ = 1e6, optional YaRN), SwiGLU MLP, untied head
(4B ties it).

MI355X execution path (one decoder layer):
  rms_norm → fused q|k|v NF4/bf16 GEMM with LoRA K-slice → q/k-norm+RoPE kernel →
  flash attention (GQA, causal) → o_proj GEMM with the residual add in its epilogue →
  rms_norm → fused gate|up GEMM → SwiGLU kernel → down GEMM (+residual) ;
  final norm → chunked LM-head + cross-entropy kernel (never materialises [T, V] fp32).
"""
from __future__ import annotations

import dataclasses
import json
import math
import os

import torch
import torch.nn as nn

from ..ops import reference as ref
from ..ops.activation import swiglu_fused
from ..ops.mlp import fusable as mlp_fusable, swiglu_mlp
from ..ops.attention import flash_attention, flash_attention_prefix
from ..ops.decode import decode_attention_append
from ..ops.linear import checkpoint as lora_checkpoint
from ..ops.loss import fused_linear_cross_entropy, shift_labels
from ..ops.norm import RMSNorm, rms_norm, rms_norm_residual
from ..ops.rope import apply_rope, qk_norm_rope
from ..parallel.tensor_parallel import tp_all_reduce
from ..peft.lora import LoraLayer, base_of
from ..quant.int4 import Int4Linear
from ..ops.embedding import Embedding
from .common import CausalLMOutput, FusedProjection, KVCache, PackedPrefill, _leaf_linear, can_fuse, project

# the SwiGLU MLP through ops/mlp.py's fused GEMM-epilogue kernels when it carries no adapters (the GPU tests
# switch this off to check the fused block against separate projections + activation kernels)
_FUSED_MLP = True


@dataclasses.dataclass
class Qwen3Config:
    vocab_size: int = 151936
    hidden_size: int = 4096
    intermediate_size: int = 12288
    num_hidden_layers: int = 36
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    head_dim: int = 128
    rms_norm_eps: float = 1e-6
    rope_theta: float = 1_000_000.0
    rope_scaling: dict | None = None
    max_position_embeddings: int = 40960
    tie_word_embeddings: bool = False
    attention_dropout: float = 0.0
    bos_token_id: int = 151643
    eos_token_id: int = 151645
    pad_token_id: int | None = None
    torch_dtype: str = "bfloat16"
    model_type: str = "qwen3"
    use_cache: bool = True
    attention_bias: bool = False      # Qwen2 (DeepSeek-R1-Distill-Qwen) has q/k/v biases
    qk_norm: bool = True              # Qwen3 per-head q/k RMSNorm; Qwen2 has none

    @classmethod
    def from_dict(cls, d: dict) -> "Qwen3Config":
        fields = {f.name for f in dataclasses.fields(cls)}
        kw = {k: v for k, v in d.items() if k in fields}
        if d.get("model_type") == "qwen2":         # DeepSeek-R1-Distill-Qwen-*: biased qkv, no qk-norm
            kw.setdefault("attention_bias", True)
            kw["qk_norm"] = False
        if "head_dim" not in d and "hidden_size" in d and "num_attention_heads" in d:
            kw["head_dim"] = d["hidden_size"] // d["num_attention_heads"]
        if "rope_parameters" in d and isinstance(d["rope_parameters"], dict):   # transformers>=5 layout
            rp = d["rope_parameters"]
            kw.setdefault("rope_theta", rp.get("rope_theta", cls.rope_theta))
            if rp.get("rope_type", "default") not in ("default", None):
                kw.setdefault("rope_scaling", rp)
        return cls(**kw)

    @classmethod
    def from_pretrained(cls, path: str) -> "Qwen3Config":
        with open(os.path.join(path, "config.json")) as f:
            return cls.from_dict(json.load(f))

    def to_dict(self) -> dict:
        d = dataclasses.asdict(self)
        d["architectures"] = ["Qwen2ForCausalLM" if self.model_type == "qwen2" else "Qwen3ForCausalLM"]
        return d

    def num_params(self) -> int:
        h, f, L = self.hidden_size, self.intermediate_size, self.num_hidden_layers
        d, hq, hkv = self.head_dim, self.num_attention_heads, self.num_key_value_heads
        attn = h * hq * d * 2 + h * hkv * d * 2 + (2 * d if self.qk_norm else 0)
        attn += (hq + 2 * hkv) * d if self.attention_bias else 0
        mlp = 3 * h * f
        emb = self.vocab_size * h * (1 if self.tie_word_embeddings else 2)
        return L * (attn + mlp + 2 * h) + emb + h


# [ext] public HF configs
PRESETS: dict[str, dict] = {
    "qwen3-8b": dict(hidden_size=4096, intermediate_size=12288, num_hidden_layers=36,
                     num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=40960),
    "qwen3-14b": dict(hidden_size=5120, intermediate_size=17408, num_hidden_layers=40,
                      num_attention_heads=40, num_key_value_heads=8, max_position_embeddings=40960),
    "qwen3-4b": dict(hidden_size=2560, intermediate_size=9728, num_hidden_layers=36,
                     num_attention_heads=32, num_key_value_heads=8, tie_word_embeddings=True,
                     max_position_embeddings=40960),
    "deepseek-r1-0528-qwen3-8b": dict(hidden_size=4096, intermediate_size=12288, num_hidden_layers=36,
                                      num_attention_heads=32, num_key_value_heads=8,
                                      max_position_embeddings=131072,
                                      rope_scaling={"rope_type": "yarn", "factor": 4.0,
                                                    "original_max_position_embeddings": 32768}),
    # Qwen2 architecture (biased q/k/v, no qk-norm): Scripts/inference/*, Scripts/fine-tuning/01-04
    "deepseek-r1-distill-qwen-1.5b": dict(vocab_size=151936, hidden_size=1536, intermediate_size=8960,
                                          num_hidden_layers=28, num_attention_heads=12, num_key_value_heads=2,
                                          head_dim=128, rope_theta=10000.0, max_position_embeddings=131072,
                                          bos_token_id=151646, eos_token_id=151643, model_type="qwen2",
                                          attention_bias=True, qk_norm=False),
    # small random-init configs for CPU tests / smoke
    "qwen3-tiny": dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, head_dim=32,
                       max_position_embeddings=512),
    "qwen3-small": dict(vocab_size=4096, hidden_size=1024, intermediate_size=3072, num_hidden_layers=4,
                        num_attention_heads=8, num_key_value_heads=4, head_dim=128,
                        max_position_embeddings=4096),
    "qwen2-tiny": dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, head_dim=32, max_position_embeddings=512,
                       rope_theta=10000.0, model_type="qwen2", attention_bias=True, qk_norm=False),
}


def qwen3_config(name: str, **overrides) -> Qwen3Config:
    kw = dict(PRESETS[name])
    kw.update(overrides)
    return Qwen3Config(**kw)


class Qwen3Attention(nn.Module):
    def __init__(self, cfg: Qwen3Config, layer_idx: int):
        super().__init__()
        self.cfg, self.layer_idx = cfg, layer_idx
        h, d = cfg.hidden_size, cfg.head_dim
        self.hq, self.hkv, self.d = cfg.num_attention_heads, cfg.num_key_value_heads, d
        ab = cfg.attention_bias
        self.q_proj = nn.Linear(h, self.hq * d, bias=ab)
        self.k_proj = nn.Linear(h, self.hkv * d, bias=ab)
        self.v_proj = nn.Linear(h, self.hkv * d, bias=ab)
        self.o_proj = nn.Linear(self.hq * d, h, bias=False)
        self.tp_group, self.tp_rank = None, 0        # set by parallel.tensor_parallel
        if cfg.qk_norm:
            self.q_norm = RMSNorm(d, cfg.rms_norm_eps)
            self.k_norm = RMSNorm(d, cfg.rms_norm_eps)
        else:
            self.q_norm = self.k_norm = None
        self._qkv: FusedProjection | None = None

    def fuse(self):
        mods = [self.q_proj, self.k_proj, self.v_proj]
        self._qkv = FusedProjection(mods) if can_fuse(mods) else None

    def forward(self, x, cos, sin, B, S, residual=None, cache: KVCache | None = None, start: int = 0,
                kv_lens=None):
        tr = self.training
        qkv = project([self.q_proj, self.k_proj, self.v_proj], x, None, tr, self._qkv)
        if self.q_norm is not None:
            q, k, v = qk_norm_rope(qkv, self.q_norm.weight, self.k_norm.weight, cos, sin,
                                   self.hq, self.hkv, self.d, self.cfg.rms_norm_eps)
        else:   # Qwen2: RoPE only
            T = qkv.shape[0]
            nq, nk = self.hq * self.d, self.hkv * self.d
            q = apply_rope(qkv[:, :nq].reshape(T, self.hq, self.d), cos, sin).reshape(T, nq)
            k = apply_rope(qkv[:, nq:nq + nk].reshape(T, self.hkv, self.d), cos, sin).reshape(T, nk)
            v = qkv[:, nq + nk:]
        if cache is None:
            o = flash_attention(q, k, v, B, S, self.hq, self.hkv, self.d, causal=True, kv_lens=kv_lens)
        elif isinstance(cache, PackedPrefill):
            o = cache.attend(self.layer_idx, q, k, v, self.hq, self.hkv, self.d, flash_attention)
        elif cache.pos is not None and S == 1:
            # decode: append at each row's own position, split-K attention over the cache
            o = decode_attention_append(q.reshape(B, -1), k.reshape(B, -1), v.reshape(B, -1), cache.k[self.layer_idx],
                                        cache.v[self.layer_idx], cache.pos, self.hq, self.hkv, self.d,
                                        max_len=cache.max_len)
        else:
            kc, vc = cache.update(self.layer_idx, k.reshape(B, S, -1), v.reshape(B, S, -1), start)
            if start == 0:   # prefill: same fused kernel as training (causal + per-row key lengths)
                o = flash_attention(q, k.reshape(B * S, -1), v.reshape(B * S, -1), B, S, self.hq, self.hkv, self.d,
                                    causal=True, kv_lens=kv_lens)
            else:   # chunked / suffix prefill: the new queries sit at start.. over the cache prefix
                c = cache.k[self.layer_idx]
                o = flash_attention_prefix(q, c, cache.v[self.layer_idx], B, S, start + S, self.hq, self.hkv,
                                           self.d, q_offs=start, kv_lens=kv_lens, kv_rows=c.shape[1])
        if self.tp_group is None:
            return project([self.o_proj], o, residual, tr)
        # row-parallel o_proj: partial sums + the residual on rank 0 only, then one all-reduce
        return tp_all_reduce(project([self.o_proj], o, residual if self.tp_rank == 0 else None, tr), self.tp_group)


class Qwen3MLP(nn.Module):
    def __init__(self, cfg: Qwen3Config):
        super().__init__()
        h, f = cfg.hidden_size, cfg.intermediate_size
        self.gate_proj = nn.Linear(h, f, bias=False)
        self.up_proj = nn.Linear(h, f, bias=False)
        self.down_proj = nn.Linear(f, h, bias=False)
        self._gu: FusedProjection | None = None
        self.tp_group, self.tp_rank = None, 0        # set by parallel.tensor_parallel

    def fuse(self):
        mods = [self.gate_proj, self.up_proj]
        self._gu = FusedProjection(mods) if can_fuse(mods) else None

    def _fused_bases(self, x):
        """(gate|up base, down base) when the whole block can run as the epilogue-fused SwiGLU
        MLP (ops/mlp.py): fused gate|up, no adapters or TP on the block, bias-free frozen bases."""
        if self._gu is None or self.tp_group is not None or not _FUSED_MLP:
            return None
        mods = (self.gate_proj, self.up_proj, self.down_proj)
        if any((isinstance(m, LoraLayer) and not m.merged) or getattr(_leaf_linear(m), "_mlora", None) is not None
               for m in mods):
            return None
        if isinstance(_leaf_linear(self.down_proj), Int4Linear):
            return None     # W4A16 runs as separate projections (base_of would dequantise the weight)
        down_base, down_bias = base_of(self.down_proj)
        if self._gu.bias is not None or down_bias is not None:
            return None
        leaf = _leaf_linear(self.gate_proj)
        if not mlp_fusable(x, self._gu.base, down_base, leaf.out_features, leaf.in_features):
            return None
        return self._gu.base, down_base

    def forward(self, x, residual=None):
        tr = self.training
        bases = self._fused_bases(x)
        if bases is not None:
            return swiglu_mlp(x, bases[0], bases[1], residual)
        gu = project([self.gate_proj, self.up_proj], x, None, tr, self._gu)
        if self.tp_group is None:
            return project([self.down_proj], swiglu_fused(gu), residual, tr)
        y = project([self.down_proj], swiglu_fused(gu), residual if self.tp_rank == 0 else None, tr)
        return tp_all_reduce(y, self.tp_group)


class Qwen3DecoderLayer(nn.Module):
    def __init__(self, cfg: Qwen3Config, layer_idx: int):
        super().__init__()
        self.self_attn = Qwen3Attention(cfg, layer_idx)
        self.mlp = Qwen3MLP(cfg)
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)

    def forward(self, x, cos, sin, B, S, cache=None, start=0, kv_lens=None):
        xn, skip = rms_norm_residual(x, self.input_layernorm.weight, self.input_layernorm.eps)
        h = self.self_attn(xn, cos, sin, B, S, residual=skip, cache=cache, start=start, kv_lens=kv_lens)
        hn, skip = rms_norm_residual(h, self.post_attention_layernorm.weight, self.post_attention_layernorm.eps)
        return self.mlp(hn, residual=skip)


class Qwen3Model(nn.Module):
    def __init__(self, cfg: Qwen3Config):
        super().__init__()
        self.cfg = cfg
        self.embed_tokens = Embedding(cfg.vocab_size, cfg.hidden_size)
        self.layers = nn.ModuleList([Qwen3DecoderLayer(cfg, i) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        inv, attn_factor = ref.rope_inv_freq(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling)
        self.register_buffer("inv_freq", inv, persistent=False)
        self.attn_factor = attn_factor
        self.gradient_checkpointing = False
        self.ckpt_kwargs: dict = {}      # use_reentrant / policy (ops/linear.py checkpoint)
        self.pp = None          # parallel.pipeline_parallel stage link (inference PP), else None
        self._rope_cache: dict = {}   # (B, S, inv_freq, factor) -> (cos, sin) for positions 0 .. S-1

    def rope(self, position_ids: torch.Tensor):
        ang = position_ids.reshape(-1).float()[:, None] * self.inv_freq[None, :]
        return (torch.cos(ang) * self.attn_factor).contiguous(), (torch.sin(ang) * self.attn_factor).contiguous()

    def forward(self, input_ids, position_ids=None, cache: KVCache | None = None, kv_lens=None):
        B, S = input_ids.shape
        start = cache.len if cache is not None else 0
        decoding = cache is not None and cache.pos is not None and S == 1
        if position_ids is None and not decoding and start == 0:
            # positions 0 .. S-1 (every training step, every fresh prefill): the cos / sin tables depend only on
            # (B, S) — computed once instead of ~7 small launches + their host time at the head of every step
            # (inv_freq's version: an in-place rescale re-keys; inference-mode tables never serve autograd)
            key = (B, S, self.inv_freq.data_ptr(), self.inv_freq._version, str(input_ids.device), self.attn_factor,
                   torch.is_inference_mode_enabled())
            cs = self._rope_cache.get(key)
            if cs is None:
                if len(self._rope_cache) >= 8:
                    self._rope_cache.clear()
                cs = self.rope(torch.arange(S, device=input_ids.device).expand(B, S))
                self._rope_cache[key] = cs
            cos, sin = cs
        else:
            if position_ids is None:
                position_ids = cache.pos[:, None] if decoding else \
                    torch.arange(start, start + S, device=input_ids.device).expand(B, S)
            cos, sin = self.rope(position_ids)
        x = self.embed_tokens(input_ids).reshape(B * S, -1)
        if self.pp is not None:
            x = self.pp.enter(x)        # stages > 0: the previous stage's hidden states
        for layer in self.layers:
            if self.gradient_checkpointing and self.training and cache is None:
                x = lora_checkpoint(layer, x, cos, sin, B, S, None, 0, kv_lens, **self.ckpt_kwargs)
            else:
                x = layer(x, cos, sin, B, S, cache, start, kv_lens)
        if self.pp is not None:
            x = self.pp.exit(x)         # hand to the next stage; every stage gets the last one's output
        if decoding:
            cache.pos += 1
        elif cache is not None:
            cache.len = start + S
        return rms_norm(x, self.norm.weight, self.norm.eps)


class Qwen3ForCausalLM(nn.Module):
    def __init__(self, cfg: Qwen3Config):
        super().__init__()
        self.config = cfg
        self.model = Qwen3Model(cfg)
        self.lm_head = nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False)
        if cfg.tie_word_embeddings:
            self.lm_head.weight = self.model.embed_tokens.weight

    # -------------------------------------------------------------- construction
    @classmethod
    def from_config(cls, cfg: Qwen3Config, dtype=torch.bfloat16, device=None, init_std: float = 0.02,
                    seed: int | None = 0) -> "Qwen3ForCausalLM":
        """Random-init (synthetic benchmark weights, no checkpoint download)."""
        if seed is not None:
            torch.manual_seed(seed)
        with torch.device(device or "cpu"):
            m = cls(cfg)
        m.to(dtype)
        with torch.no_grad():
            for n, p in m.named_parameters():
                if p.dim() == 2:
                    p.normal_(0.0, init_std)
        return m

    def gradient_checkpointing_enable(self, gradient_checkpointing_kwargs=None):
        """HF's API (``Fine-Tuning/qwen3-8b-qlora-dist.py:162-163``): ``use_reentrant`` selects torch's
        checkpoint form; ``policy`` ("full" default = HF's whole-layer recompute / "selective" = keep the GEMM
        outputs, ≈ 78 MB more per layer per 1024 tokens) is this framework's recompute policy (ops/linear.py
        ``checkpoint``).  Unknown keys raise."""
        kw = dict(gradient_checkpointing_kwargs or {})
        bad = set(kw) - {"use_reentrant", "policy"}
        if bad:
            raise ValueError(f"gradient_checkpointing_kwargs: unsupported keys {sorted(bad)}")
        self.model.gradient_checkpointing = True
        self.model.ckpt_kwargs = kw

    def gradient_checkpointing_disable(self):
        self.model.gradient_checkpointing = False

    def enable_input_require_grads(self):
        pass  # inputs of our fused ops never need requires_grad for checkpointing

    def fuse_projections(self):
        """Fuse q|k|v and gate|up into single GEMMs (call after quantisation / LoRA)."""
        for layer in self.model.layers:
            layer.self_attn.fuse()
            layer.mlp.fuse()
        return self

    def invalidate_fusion(self):
        for layer in self.model.layers:
            layer.self_attn._qkv = None
            layer.mlp._gu = None

    # -------------------------------------------------------------- forward
    def forward(self, input_ids, attention_mask=None, labels=None, position_ids=None,
                past_key_values: KVCache | None = None, use_cache: bool = False,
                return_logits: bool | None = None, num_micro_batches: int = 1, **_) -> CausalLMOutput:
        """``num_micro_batches=G`` treats the batch as G gradient-accumulation micro-batches
        run in ONE pass: the loss is the mean of the G per-micro-batch mean losses, exactly
        what sequential accumulation of ``loss_i / G`` produces (same gradient)."""
        B, S = input_ids.shape
        kv_lens = None
        if attention_mask is not None and (past_key_values is None or
                                           (past_key_values.len == 0 and past_key_values.pos is None)):
            am = attention_mask.to(torch.int32)
            lens = am.sum(1).to(torch.int32)
            if torch.equal(am, (torch.arange(S, device=am.device)[None] < lens[:, None]).int()):
                kv_lens = lens                     # right padding: exact via per-row key length
        h = self.model(input_ids, position_ids, past_key_values, kv_lens)
        loss = logits = None
        if labels is not None:
            tgt = shift_labels(labels).reshape(-1)
            G = num_micro_batches
            if G > 1:
                assert B % G == 0, "batch must split into equal micro-batches"
            loss = fused_linear_cross_entropy(h, self.lm_head.weight, tgt, groups=G)
            if return_logits:
                logits = (h @ self.lm_head.weight.t()).view(B, S, -1)
        else:
            logits = (h @ self.lm_head.weight.t()).view(B, S, -1)
        return CausalLMOutput(loss=loss, logits=logits, past_key_values=past_key_values)

    @torch.no_grad()
    def generate(self, input_ids=None, attention_mask=None, generation_config=None, streamer=None, **kw):
        """HF-style ``generate`` (KV cache, greedy / temperature / top-k / top-p / repetition
        penalty); see :func:`llm_in_practise_amd.infer.generate.generate`."""
        from ..infer.generate import generate
        return generate(self, input_ids, attention_mask, generation_config, streamer=streamer, **kw)

    # -------------------------------------------------------------- checkpoint IO
    def load_hf_state_dict(self, sd: dict[str, torch.Tensor], strict: bool = False):
        own = self.state_dict()
        missing = [k for k in own if k not in sd and "inv_freq" not in k]
        with torch.no_grad():
            for k, v in sd.items():
                if k in own:
                    own[k].copy_(v.to(own[k].dtype))
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:8]}")
        return missing

    @classmethod
    def from_pretrained(cls, path: str, dtype=torch.bfloat16, device=None, quantization_config=None,
                        rope_scaling="keep", **_) -> "Qwen3ForCausalLM":
        """Load ``config.json`` + ``*.safetensors`` shards from a local HF-layout dir.
        ``quantization_config`` (``BitsAndBytesConfig``-like, ``load_in_4bit``) quantises each
        linear to NF4 as it is loaded (on the GPU kernel when ``device`` is cuda)."""
        from safetensors import safe_open
        cfg = Qwen3Config.from_pretrained(path)
        if rope_scaling != "keep":
            cfg.rope_scaling = rope_scaling          # E7 passes rope_scaling=None
        with torch.device("meta"):
            m = cls(cfg)
        m.to_empty(device=device or "cpu")
        m.to(dtype)
        files = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
        sd = {}
        for f in files:
            with safe_open(os.path.join(path, f), framework="pt", device="cpu") as fh:
                for k in fh.keys():
                    sd[k] = fh.get_tensor(k)
        m.load_hf_state_dict(sd)
        inv, af = ref.rope_inv_freq(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling)
        m.model.inv_freq = inv.to(device or "cpu")
        m.model.attn_factor = af
        if cfg.tie_word_embeddings:
            m.lm_head.weight = m.model.embed_tokens.weight
        if quantization_config is not None and getattr(quantization_config, "load_in_4bit", False):
            from ..peft.lora import quantize_model_nf4
            quantize_model_nf4(m, double_quant=quantization_config.bnb_4bit_use_double_quant,
                               compute_dtype=quantization_config.bnb_4bit_compute_dtype)
        return m

    def save_pretrained(self, path: str, max_shard_bytes: int = 4 << 30):
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        sd = {k: v.detach().cpu().contiguous() for k, v in self.state_dict().items()
              if "inv_freq" not in k}
        if self.config.tie_word_embeddings:
            sd.pop("lm_head.weight", None)
        shards, cur, size = [], {}, 0
        for k, v in sd.items():
            nb = v.numel() * v.element_size()
            if cur and size + nb > max_shard_bytes:
                shards.append(cur)
                cur, size = {}, 0
            cur[k] = v
            size += nb
        shards.append(cur)
        index = {}
        for i, sh in enumerate(shards):
            name = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors" if len(shards) > 1 else "model.safetensors"
            save_file(sh, os.path.join(path, name), metadata={"format": "pt"})
            index.update({k: name for k in sh})
        if len(shards) > 1:
            with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
                json.dump({"metadata": {}, "weight_map": index}, f, indent=1)
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(self.config.to_dict(), f, indent=2)


class BitsAndBytesConfig:
    """Argument-compatible stand-in for ``transformers.BitsAndBytesConfig`` (NF4 only)."""

    def __init__(self, load_in_4bit=False, bnb_4bit_compute_dtype=torch.bfloat16, bnb_4bit_quant_type="nf4",
                 bnb_4bit_use_double_quant=False, bnb_4bit_quant_storage=torch.uint8, **_):
        assert bnb_4bit_quant_type == "nf4", "only NF4 is implemented (the reference uses nf4)"
        self.load_in_4bit = load_in_4bit
        self.bnb_4bit_compute_dtype = bnb_4bit_compute_dtype
        self.bnb_4bit_quant_type = bnb_4bit_quant_type
        self.bnb_4bit_use_double_quant = bnb_4bit_use_double_quant
        self.bnb_4bit_quant_storage = bnb_4bit_quant_storage
