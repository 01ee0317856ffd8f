"""Affine 4-bit weight-only quantisation, W4A16.

Storage (one canonical layout for every producer — RTN, GPTQ, AWQ — and every on-disk format):
``codes`` uint8 [N, K/2] with the HIGH nibble holding the even k (the NF4 convention, so the
same fragment-native repacker feeds the MFMA kernel), unsigned q ∈ [0, 15]; ``scales`` fp32
[N, K/g]; ``zeros`` uint8 [N, K/g] (8 for symmetric).  Dequant: ``w = (q − z)·s``.

Kernels (dispatch in :func:`int4_linear`): ``gemv.hip`` (M ≤ 2, weight-streaming GEMV, ``q·s + b``
with ``b = −z·s`` per group), ``w4mm.hip`` (M ≤ 32: the MFMA sums x·(128+q) from byte-permuted
codes, the group's scale and zero fold after it), ``gemm4w.hip`` W4 = 2 (larger M: the codes expanded
through a per-block (q − z)·s table into the bf16 B image of the hand-written GEMM).

On-disk formats (converters below; exact bit layouts documented per function — no reference
checkpoint ships with the reference repo, so byte-level parity is *unpinned* and covered by
round-trip tests):
  * compressed-tensors ``pack-quantized`` (llm-compressor ``oneshot`` output, F2/F3/F4):
    ``weight_packed`` int32 [N, K/8], ``weight_scale`` [N, K/g], ``weight_zero_point`` int32
    [N/8, K/g] (asymmetric), ``weight_shape``;
  * GPTQ (GPTQModel / AutoGPTQ v1, F1): ``qweight`` int32 [K/8, N], ``qzeros`` int32 [K/g, N/8]
    (stored minus one), ``scales`` fp16 [K/g, N], ``g_idx`` int32 [K];
  * AWQ GEMM: ``qweight`` int32 [K, N/8] and ``qzeros`` [K/g, N/8] in the AWQ nibble order
    (0, 2, 4, 6, 1, 3, 5, 7), ``scales`` fp16 [K/g, N].
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn as nn


@dataclasses.dataclass
class Int4Weight:
    codes: torch.Tensor          # uint8 [N, K/2]
    scales: torch.Tensor         # fp32 [N, K/g]
    zeros: torch.Tensor          # uint8 [N, K/g]
    shape: tuple
    group_size: int = 128
    sym: bool = False
    _gemv: tuple | None = None

    @property
    def dtype(self):
        return torch.bfloat16

    def q(self) -> torch.Tensor:
        """Unsigned codes [N, K] (int16)."""
        n, k = self.shape
        hi = (self.codes >> 4).to(torch.int16)
        lo = (self.codes & 0xF).to(torch.int16)
        return torch.stack([hi, lo], -1).reshape(n, k)

    def dequantize(self, dtype=torch.float32) -> torch.Tensor:
        n, k = self.shape
        g = self.group_size
        q = self.q().float().view(n, k // g, g)
        w = (q - self.zeros.float()[..., None]) * self.scales.float()[..., None]
        return w.view(n, k).to(dtype)

    def to(self, device):
        out = dataclasses.replace(self, codes=self.codes.to(device), scales=self.scales.to(device),
                                  zeros=self.zeros.to(device), _gemv=None)
        out.__dict__.pop("_g4w", None)
        out.__dict__.pop("_w4mm", None)
        return out

    def bias_table(self) -> torch.Tensor:
        return -(self.zeros.float() * self.scales.float())

    def kernel_ok(self) -> bool:
        n, k = self.shape
        return n % 32 == 0 and k % 64 == 0 and self.group_size % 64 == 0

    def g4w_pack(self) -> tuple:
        """(codes, scale_t, zero_t) — the affine-int4 B operand of the hand-written gemm4w GEMM (the NF4
        dequant-GEMM's kernel with a (q − z)·s table): the codes re-tiled like NF4 (same nibble
        convention) and fp32 [K/64, N] scale / zero tables, each group's value repeated per 64-block."""
        c = self.__dict__.get("_g4w")
        if c is None:
            from ..ops._native import native
            n, k = self.shape
            rep = self.group_size // 64
            codes = native().g4w_pack(self.codes.contiguous(), n, k)
            st = self.scales.float().repeat_interleave(rep, dim=1).t().contiguous()
            zt = self.zeros.float().repeat_interleave(rep, dim=1).t().contiguous()
            c = (codes, st, zt)
            self.__dict__["_g4w"] = c
        return c

    def g4w_ok(self) -> bool:
        n, k = self.shape
        return n % 64 == 0 and k % 64 == 0 and self.group_size % 64 == 0

    def w4mm_table(self) -> torch.Tensor:
        """fp32 [N, K/g, 2] = (scale, bias − 128·scale) for the w4mm kernel (csrc/kernels/w4mm.hip: the
        MFMA sums x·(128+q), the group folds as s·G + (b − 128·s)·Σx); cached."""
        t = self.__dict__.get("_w4mm")
        if t is None:
            s = self.scales.float()
            t = torch.stack([s, self.bias_table() - 128.0 * s], -1).contiguous()
            self.__dict__["_w4mm"] = t
        return t

    def gemv_tables(self):
        if self._gemv is None:
            self._gemv = (self.scales.float().contiguous(), self.bias_table().contiguous())
        return self._gemv

    def nbytes(self) -> int:
        return self.codes.numel() + self.scales.numel() * 2 + self.zeros.numel() // 2


def pack_codes(q: torch.Tensor) -> torch.Tensor:
    """q [N, K] (0..15) → uint8 [N, K/2], high nibble = even k."""
    q = q.to(torch.uint8)
    return ((q[:, 0::2] << 4) | q[:, 1::2]).contiguous()


def quant_params(w: torch.Tensor, bits: int = 4, sym: bool = False):
    """Per-row (last dim reduced) scale/zero for ``w [..., g]`` — the min/max quantiser used by
    RTN, GPTQ's group statistics and AWQ."""
    qmax = 2 ** bits - 1
    if sym:
        amax = w.abs().amax(-1).clamp(min=1e-8)
        scale = amax / ((qmax - 1) / 2)            # 7 for int4: q − 8 ∈ [−7, 7] (+ −8 unused)
        zero = torch.full_like(scale, (qmax + 1) // 2)
    else:
        wmin = w.amin(-1).clamp(max=0)
        wmax = w.amax(-1).clamp(min=0)
        scale = ((wmax - wmin) / qmax).clamp(min=1e-8)
        zero = torch.round(-wmin / scale).clamp(0, qmax)
    return scale, zero


def quantize_rtn(w: torch.Tensor, group_size: int = 128, sym: bool = False) -> Int4Weight:
    """Round-to-nearest W4A16 (the baseline the calibrated methods improve on)."""
    n, k = w.shape
    assert k % group_size == 0 and k % 2 == 0
    wg = w.detach().float().view(n, k // group_size, group_size)
    scale, zero = quant_params(wg, 4, sym)
    q = torch.clamp(torch.round(wg / scale[..., None]) + zero[..., None], 0, 15)
    return Int4Weight(pack_codes(q.view(n, k)), scale, zero.to(torch.uint8), (n, k), group_size, sym)


def from_parts(q: torch.Tensor, scales: torch.Tensor, zeros: torch.Tensor, group_size: int,
               sym: bool = False) -> Int4Weight:
    n, k = q.shape
    return Int4Weight(pack_codes(q), scales.float().contiguous(), zeros.to(torch.uint8).contiguous(), (n, k),
                      group_size, sym)


# ============================================================================ on-disk formats
def _pack_int32(v: torch.Tensor, dim: int, order=tuple(range(8))) -> torch.Tensor:
    """Pack 8 consecutive 4-bit values along ``dim`` into int32 (value order[i] at bits 4i)."""
    v = v.to(torch.int64).movedim(dim, -1)
    sh = v.shape
    v = v.reshape(*sh[:-1], sh[-1] // 8, 8)[..., list(order)]
    out = torch.zeros(v.shape[:-1], dtype=torch.int64)
    for i in range(8):
        out |= (v[..., i] & 0xF) << (4 * i)
    out = torch.where(out >= 2 ** 31, out - 2 ** 32, out).to(torch.int32)
    return out.movedim(-1, dim).contiguous()


def _unpack_int32(p: torch.Tensor, dim: int, order=tuple(range(8))) -> torch.Tensor:
    p = p.to(torch.int64).movedim(dim, -1) & 0xFFFFFFFF
    vals = torch.stack([(p >> (4 * i)) & 0xF for i in range(8)], -1)
    inv = [0] * 8
    for i, o in enumerate(order):
        inv[o] = i
    vals = vals[..., inv]
    vals = vals.reshape(*p.shape[:-1], p.shape[-1] * 8)
    return vals.movedim(-1, dim).contiguous()


AWQ_ORDER = (0, 2, 4, 6, 1, 3, 5, 7)


def to_compressed_tensors(w: Int4Weight, scale_dtype=torch.bfloat16) -> dict:
    """compressed-tensors ``pack-quantized``: signed q' = q − 8 ∈ [−8, 7] stored as q' + 8 (= q),
    8 per int32 along K (little-endian nibbles); zero points likewise shifted, packed along N."""
    n, k = w.shape
    d = {"weight_packed": _pack_int32(w.q().cpu(), 1), "weight_scale": w.scales.cpu().to(scale_dtype),
         "weight_shape": torch.tensor([n, k], dtype=torch.int64)}
    if not w.sym:
        d["weight_zero_point"] = _pack_int32(w.zeros.cpu().to(torch.int64), 0)
    return d


def from_compressed_tensors(d: dict, group_size: int, sym: bool | None = None) -> Int4Weight:
    n, k = [int(x) for x in d["weight_shape"].tolist()]
    q = _unpack_int32(d["weight_packed"], 1)[:, :k]
    if "weight_zero_point" in d and d["weight_zero_point"].numel() > 1:
        z = _unpack_int32(d["weight_zero_point"], 0)[:n]
        sym = False if sym is None else sym
    else:
        z = torch.full((n, k // group_size), 8, dtype=torch.int64)
        sym = True if sym is None else sym
    return from_parts(q, d["weight_scale"].float(), z, group_size, sym)


def to_gptq(w: Int4Weight) -> dict:
    """GPTQ v1 tensors (qzeros stored minus one, the AutoGPTQ convention)."""
    n, k = w.shape
    g = w.group_size
    q = w.q().cpu().t()                                          # [K, N]
    z = (w.zeros.cpu().to(torch.int64) - 1).clamp(min=0).t()    # [K/g, N]
    return {"qweight": _pack_int32(q, 0), "qzeros": _pack_int32(z, 1),
            "scales": w.scales.cpu().t().contiguous().to(torch.float16),
            "g_idx": (torch.arange(k) // g).to(torch.int32)}


def from_gptq(d: dict, group_size: int, sym: bool = False) -> Int4Weight:
    q = _unpack_int32(d["qweight"], 0).t()                        # [N, K]
    z = (_unpack_int32(d["qzeros"], 1) + 1).t()                   # [N, K/g]
    n = q.shape[0]
    return from_parts(q, d["scales"].float().t()[:n], z[:n], group_size, sym)


def to_awq(w: Int4Weight) -> dict:
    q = w.q().cpu().t()                                          # [K, N]
    z = w.zeros.cpu().to(torch.int64).t()                        # [K/g, N]
    return {"qweight": _pack_int32(q, 1, AWQ_ORDER), "qzeros": _pack_int32(z, 1, AWQ_ORDER),
            "scales": w.scales.cpu().t().contiguous().to(torch.float16)}


def from_awq(d: dict, group_size: int) -> Int4Weight:
    q = _unpack_int32(d["qweight"], 1, AWQ_ORDER).t()
    z = _unpack_int32(d["qzeros"], 1, AWQ_ORDER).t()
    return from_parts(q, d["scales"].float().t(), z, group_size, False)


# ============================================================================ module + op
# W4A16 kernel per row count (measured on the Qwen3-8B projection shapes, profiles/r4/w4a16_w4mm.txt,
# profiles/r5/w4g_decode.txt):
#   M <= 2      gemv_w4 (csrc/kernels/gemv.hip): weight-streaming GEMV, no matrix-core padding;
#   3 .. 32     w4mm (csrc/kernels/w4mm.hip): byte-permute dequant, MFMA, per-group scale folded after it;
#   33 .. 64    w4g (w4mm.hip w4g_k): the same dequant / fold tiled for decode batches — x streamed per
#               128-deep block through LDS once per column span, codes two blocks ahead in registers;
#   65 .. 1023  gemm4w with the affine table expanded in-kernel (csrc/kernels/gemm4w_kernel.h, W4 = 2);
#   >= 1024     prefill: one HBM-speed bf16 expansion (int4_dequant_k, 6.6 TB/s) into a transient copy + the
#               gemm4w bf16 GEMM (ops/linear.py _base_gemm) — at these row counts the in-kernel table costs more
#               than the expansion (per layer at M = 2048: 708 -> 639 µs; profiles/r4/w4a16_prefill.txt);
# anything the kernels do not take: one bf16 dequantisation + torch matmul.
_W4MM_MAX = 32
_W4G_MAX = 64
_EXPAND_MIN = 1024


def int4_linear(x: torch.Tensor, w: Int4Weight, bias: torch.Tensor | None = None,
                residual: torch.Tensor | None = None) -> torch.Tensor:
    from ..ops._native import native, use_native
    shape = x.shape
    x2 = x.reshape(-1, shape[-1])
    n, k = w.shape
    r2 = residual.reshape(-1, n).contiguous() if residual is not None else None
    M = x2.shape[0]
    nat = use_native(x2) and x2.dtype == torch.bfloat16 and x2.stride(-1) == 1
    if nat and M <= 2 and w.kernel_ok():
        s, b = w.gemv_tables()
        y = native().gemv_w4(x2.contiguous(), w.codes, s, b, n, w.group_size, r2)
    elif nat and M <= _W4MM_MAX and native().w4mm_ok(M, n, k, w.group_size):
        y = native().w4mm(x2.contiguous(), w.codes, w.w4mm_table(), n, w.group_size, r2)
    elif nat and M <= _W4G_MAX and native().w4g_ok(M, n, k, w.group_size):
        y = native().w4g(x2.contiguous(), w.codes, w.w4mm_table(), n, w.group_size, r2)
    elif nat and M >= _EXPAND_MIN and k % w.group_size == 0 and w.group_size % 8 == 0:
        from ..ops.linear import _base_gemm
        s, b = w.gemv_tables()
        wb = native().int4_dequant(w.codes, s, b, n, k, w.group_size)
        y = _base_gemm(x2, wb, residual=r2)
        del wb
    elif nat and w.g4w_ok():
        codes, st, zt = w.g4w_pack()
        y = native().gemm4w(x2.contiguous(), codes, r2, 0, False, 0, 0, st, n, zt)
    else:
        y = x2 @ w.dequantize(x2.dtype).t()
        if r2 is not None:
            y = y + r2
    if bias is not None:
        y = y + bias
    return y.view(*shape[:-1], n)


class Int4Linear(nn.Module):
    """Frozen W4A16 linear (the GPTQ/AWQ ``QuantLinear`` role)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False, group_size: int = 128):
        super().__init__()
        self.in_features, self.out_features, self.group_size = in_features, out_features, group_size
        self.register_buffer("codes", torch.zeros(0, dtype=torch.uint8))
        self.register_buffer("scales", torch.zeros(0))
        self.register_buffer("zeros", torch.zeros(0, dtype=torch.uint8))
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=torch.bfloat16), requires_grad=False) if bias else None
        self.sym = False

    @classmethod
    def from_weight(cls, w: Int4Weight, bias: torch.Tensor | None = None) -> "Int4Linear":
        m = cls(w.shape[1], w.shape[0], bias is not None, w.group_size)
        m.load(w)
        if bias is not None:
            m.bias.data = bias.detach().to(torch.bfloat16)
        return m

    def load(self, w: Int4Weight):
        self.codes, self.scales, self.zeros, self.sym = w.codes, w.scales, w.zeros, w.sym
        self.group_size = w.group_size
        self.__dict__.pop("_int4_cache", None)

    @property
    def int4(self) -> Int4Weight:
        c = self.__dict__.get("_int4_cache")
        if c is None or c.codes is not self.codes:
            c = Int4Weight(self.codes, self.scales, self.zeros, (self.out_features, self.in_features),
                           self.group_size, self.sym)
            self.__dict__["_int4_cache"] = c
        return c

    @property
    def weight(self):
        return self.int4.dequantize(torch.bfloat16)

    def forward(self, x):
        return int4_linear(x.to(torch.bfloat16) if x.is_cuda else x, self.int4, self.bias)

    def extra_repr(self):
        return f"in={self.in_features}, out={self.out_features}, w4a16 g{self.group_size}{' sym' if self.sym else ''}"
