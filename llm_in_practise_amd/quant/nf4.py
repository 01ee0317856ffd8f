"""NF4 (4-bit NormalFloat) weight quantisation for QLoRA — no bitsandbytes.

Reference usage: ``BitsAndBytesConfig(load_in_4bit=True, bnb_4bit_quant_type="nf4",
bnb_4bit_use_double_quant=True, bnb_4bit_compute_dtype=torch.bfloat16)``
(``Fine-Tuning/qwen3-8b-qlora.py:93-100``).

Format (the bitsandbytes layout [ext], re-derived, kept kernel-friendly):
  * blocks of ``blocksize`` (64) consecutive elements of the row-major weight get one
    ``absmax``; each element stores the index of the nearest NF4 code of ``x/absmax``;
  * two codes per byte, the FIRST element in the HIGH nibble;
  * double quant: ``absmax - offset`` is quantised blockwise (256 absmax per group) to
    8 bits with the signed dynamic map; ``offset = mean(absmax)`` of the tensor.

MI355X-specific choice: ``offset`` is stored per 256-absmax *group* (same value for all
groups of one tensor).  That lets the kernels treat a row-concatenation of several
quantised tensors (fused q|k|v or gate|up weights) as ONE quantised matrix with no
per-tensor metadata — the fused NF4 GEMM reads ``qabsmax``, ``absmax2`` and ``offset``
by group index only.
"""
from __future__ import annotations

import dataclasses
import functools

import torch

# bitsandbytes NF4 table (quantiles of N(0,1) rescaled to [-1, 1]) [ext]
NF4_CODE = [
    -1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
    -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
    0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
    0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0,
]
DQ_GROUP = 256  # absmax values per double-quant group


@functools.lru_cache(maxsize=None)
def nf4_code(device: str = "cpu") -> torch.Tensor:
    return torch.tensor(NF4_CODE, dtype=torch.float32, device=device)


def create_dynamic_map(signed: bool = True, max_exponent_bits: int = 7, total_bits: int = 8) -> torch.Tensor:
    """Signed dynamic (exponent + linear fraction) 8-bit map used for double quant [ext]."""
    data: list[float] = []
    non_sign_bits = total_bits - 1
    additional_items = 2 ** (non_sign_bits - max_exponent_bits) - 1
    i = 0
    for i in range(max_exponent_bits):
        fraction_items = int(2 ** (i + non_sign_bits - max_exponent_bits) + 1 if signed
                             else 2 ** (i + non_sign_bits - max_exponent_bits + 1) + 1)
        boundaries = torch.linspace(0.1, 1, fraction_items, dtype=torch.float64)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
        if signed:
            data += (-(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
    if additional_items > 0:
        boundaries = torch.linspace(0.1, 1, additional_items + 1, dtype=torch.float64)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
        if signed:
            data += (-(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
    data.append(0.0)
    data.append(1.0)
    data += [0.0] * (2 ** total_bits - len(data))
    data.sort()
    return torch.tensor(data, dtype=torch.float32)


@functools.lru_cache(maxsize=None)
def dynamic_code(device: str = "cpu") -> torch.Tensor:
    return create_dynamic_map().to(device)


def _nearest(values: torch.Tensor, code: torch.Tensor, chunk: int = 1 << 22) -> torch.Tensor:
    """Index of the nearest entry of a sorted ``code`` for each value (midpoint search)."""
    mids = (code[1:] + code[:-1]) * 0.5
    out = torch.empty(values.shape, dtype=torch.uint8, device=values.device)
    flat, oflat = values.reshape(-1), out.view(-1)
    for s in range(0, flat.numel(), chunk):
        oflat[s:s + chunk] = torch.bucketize(flat[s:s + chunk], mids).to(torch.uint8)
    return out


@dataclasses.dataclass
class NF4Weight:
    """A quantised ``[out_features, in_features]`` weight."""
    codes: torch.Tensor            # uint8 [N, K//2]   (high nibble = even k)
    absmax: torch.Tensor | None    # fp32 [N*K//bs]     (when not double-quantised)
    qabsmax: torch.Tensor | None   # uint8 [N*K//bs]    (double quant)
    absmax2: torch.Tensor | None   # fp32 [groups]
    offset: torch.Tensor | None    # fp32 [groups]
    shape: tuple[int, int]
    blocksize: int = 64
    dtype: torch.dtype = torch.bfloat16   # compute / dequant dtype

    @property
    def double_quant(self) -> bool:
        return self.qabsmax is not None

    @property
    def device(self) -> torch.device:
        return self.codes.device

    def nbytes(self) -> int:
        n = self.codes.numel()
        for t in (self.absmax, self.qabsmax, self.absmax2, self.offset):
            if t is not None:
                n += t.numel() * t.element_size()
        return n

    def tensors(self) -> dict[str, torch.Tensor]:
        d = {"codes": self.codes}
        for k in ("absmax", "qabsmax", "absmax2", "offset"):
            v = getattr(self, k)
            if v is not None:
                d[k] = v
        return d

    def to(self, device) -> "NF4Weight":
        m = {f.name: getattr(self, f.name) for f in dataclasses.fields(self)}
        m = {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in m.items()}
        return NF4Weight(**m)

    def g4w_pack(self) -> tuple:
        """(codes, scales_t) — the NF4 B operand of the hand-written gemm4w GEMM (csrc/kernels/gemm4w.hip):
        the codes re-tiled to [N/64][K/64][2][64][16 B] (pack_g4w_k) and the decoded fp32 block absmax
        transposed to [K/64, N].  Same bytes as the bnb layout, permuted; built once on first use."""
        c = self.__dict__.get("_g4w")
        if c is None:
            from ..ops._native import native
            n, k = self.shape
            codes = native().g4w_pack(self.codes.contiguous(), n, k)
            sc = self.gemv_scales().reshape(n, k // 64).t().contiguous()
            c = (codes, sc)
            self.__dict__["_g4w"] = c
        return c

    def kernel_ok(self) -> bool:
        n, k = self.shape
        return self.blocksize == 64 and n % 64 == 0 and k % 64 == 0

    def gemv_scales(self) -> torch.Tensor:
        """Decoded fp32 block absmax [N, K/64] for the decode GEMV (cached)."""
        c = self.__dict__.get("_gemv_sc")
        if c is None:
            c = self.block_absmax().float().contiguous()
            self.__dict__["_gemv_sc"] = c
        return c

    def block_absmax(self) -> torch.Tensor:
        """fp32 absmax per block, decoding the double quant."""
        if self.absmax is not None:
            return self.absmax
        code = dynamic_code(str(self.codes.device))
        g = torch.arange(self.qabsmax.numel(), device=self.codes.device) // DQ_GROUP
        return code[self.qabsmax.long()] * self.absmax2[g] + self.offset[g]


def quantize_nf4(w: torch.Tensor, blocksize: int = 64, double_quant: bool = True,
                 compute_dtype: torch.dtype = torch.bfloat16) -> NF4Weight:
    """Quantise a 2-D weight to NF4 (pure PyTorch; runs on CPU or GPU)."""
    assert w.dim() == 2, "NF4 quantises 2-D linear weights"
    n, k = w.shape
    assert k % blocksize == 0 and blocksize % 2 == 0
    wf = w.detach().float().reshape(-1, blocksize)
    absmax = wf.abs().amax(dim=1).clamp_min(1e-12)
    code = nf4_code(str(w.device))
    idx = _nearest(wf / absmax[:, None], code)                  # [nb, bs] uint8
    idx = idx.view(n, k)
    codes = ((idx[:, 0::2] << 4) | idx[:, 1::2]).contiguous()
    q = NF4Weight(codes, absmax.contiguous(), None, None, None, (n, k), blocksize, compute_dtype)
    return double_quantize_absmax(q) if double_quant else q


def double_quantize_absmax(q: NF4Weight) -> NF4Weight:
    """Quantise fp32 block absmax to 8-bit dynamic codes in groups of 256 (bnb double quant)."""
    absmax = q.absmax
    nb = absmax.numel()
    offset = absmax.mean()
    centred = absmax - offset
    ng = max(1, (nb + DQ_GROUP - 1) // DQ_GROUP)
    pad = ng * DQ_GROUP - nb
    cpad = torch.cat([centred, centred.new_zeros(pad)]) if pad else centred
    grp = cpad.view(ng, -1)
    absmax2 = grp.abs().amax(dim=1).clamp_min(1e-12)
    dcode = dynamic_code(str(absmax.device))
    qabs = _nearest(grp / absmax2[:, None], dcode).view(-1)[:nb].contiguous()
    offs = offset.expand(ng).contiguous()
    return NF4Weight(q.codes, None, qabs, absmax2.contiguous(), offs, q.shape, q.blocksize, q.dtype)


def dequantize_nf4(q: NF4Weight, dtype: torch.dtype | None = None) -> torch.Tensor:
    """Pure-PyTorch dequantisation (the fp32 reference for the HIP kernels)."""
    n, k = q.shape
    code = nf4_code(str(q.device))
    hi = (q.codes >> 4).long()
    lo = (q.codes & 0xF).long()
    idx = torch.stack([hi, lo], dim=-1).view(n, k)
    vals = code[idx].view(-1, q.blocksize) * q.block_absmax()[:, None]
    return vals.view(n, k).to(dtype or q.dtype)


def concat_nf4(parts: list[NF4Weight]) -> NF4Weight:
    """Row-concatenate quantised weights (fused q|k|v, gate|up).  Exact: blocks and
    double-quant groups never straddle a part when every part's block count is a multiple
    of 256 (true for all Qwen3 shapes)."""
    k = parts[0].shape[1]
    assert all(p.shape[1] == k and p.blocksize == parts[0].blocksize for p in parts)
    dq = parts[0].double_quant
    assert all(p.double_quant == dq for p in parts)
    n = sum(p.shape[0] for p in parts)
    codes = torch.cat([p.codes for p in parts], 0)
    if dq:
        for p in parts:
            assert p.qabsmax.numel() % DQ_GROUP == 0, "part not group aligned"
        return NF4Weight(codes, None, torch.cat([p.qabsmax for p in parts]),
                         torch.cat([p.absmax2 for p in parts]), torch.cat([p.offset for p in parts]),
                         (n, k), parts[0].blocksize, parts[0].dtype)
    return NF4Weight(codes, torch.cat([p.absmax for p in parts]), None, None, None,
                     (n, k), parts[0].blocksize, parts[0].dtype)
