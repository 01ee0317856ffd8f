"""Multi-adapter LoRA kernels (csrc/kernels/lora.hip: lora_proj_m, lora_proj_cols, lora_acc_jobs, lora_dxc)
against plain fp32 PyTorch, and the model-level path against the per-adapter kernels.

BASELINE #2 (``Fine-Tuning/qwen3-8b-lora.py:128-141``: r 16 / alpha 32 / dropout 0.05 on q, k, v, o) puts
three adapters on the fused q|k|v projection and one on o; these kernels serve that case."""
import pytest
import torch

from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model, quantize_model_nf4

pytestmark = pytest.mark.gpu


def _keep(ext, M, K, p, key):
    """The counter-hash keep mask of (key, element) as bool [M, K] (what every LoRA kernel draws)."""
    return ext.dropout_fwd(torch.ones(M, K, dtype=torch.bfloat16, device="cuda"), p, key) != 0


def _unpack(bits, K):
    """keep-bit plane uint8 [M, K/8] -> bool [M, K] (bit e of byte k/8 = element 8·(k/8) + e)."""
    sh = torch.arange(8, device=bits.device, dtype=torch.uint8)
    return ((bits[..., None] >> sh) & 1).bool().reshape(bits.shape[0], K)


@pytest.mark.parametrize("M,K,ranks,ps", [(512, 1024, [16, 16, 16], [0.05, 0.05, 0.05]),
                                          (300, 2048, [16], [0.1]),
                                          (256, 512, [8, 16, 8, 16], [0.0, 0.2, 0.05, 0.0])])
def test_lora_proj_m_matches_fp32(native_ext, M, K, ranks, ps):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    As = [(torch.randn(r, K, device="cuda", generator=g) * 0.05).bfloat16() for r in ranks]
    keys = [1234 + 77 * i if p > 0 else 0 for i, p in enumerate(ps)]
    scales = [2.0, 0.5, 1.0, 1.5][:len(ranks)]
    masks = torch.empty(len(ranks), M, K // 8, dtype=torch.uint8, device="cuda")
    obs = [torch.zeros(M, r, dtype=torch.bfloat16, device="cuda") for r in ranks]
    outs = native_ext.lora_proj_m(x, As, obs, True, ps, keys, scales, masks)
    for b, (a, p) in enumerate(zip(As, ps)):
        keep = _keep(native_ext, M, K, p, keys[b]) if p > 0 else torch.ones(M, K, dtype=torch.bool, device="cuda")
        assert torch.equal(_unpack(masks[b], K), keep), b
        xd = x.float() * keep / (1 - p)
        ref = scales[b] * xd @ a.float().t()
        err = (outs[b] - ref).norm() / ref.norm()
        assert err < 5e-3, (b, float(err))
        assert ((obs[b].float() - ref).norm() / ref.norm()) < 1e-2


@pytest.mark.parametrize("M", [512, 4096])   # 4096 rows: the two-step (rank 16, >= 16 row blocks) form
def test_lora_proj_cols_and_acc_jobs_match_fp32(native_ext, M):
    g = torch.Generator(device="cuda").manual_seed(1)
    K = 1024
    ncols = [1024, 512, 512]
    c0s = [0, 1024, 1536]
    dy = torch.randn(M, sum(ncols), device="cuda", generator=g).bfloat16()
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    bts = [(torch.randn(16, n, device="cuda", generator=g) * 0.05).bfloat16() for n in ncols]
    sc = [2.0, 2.0, 0.5]
    gl = native_ext.lora_proj_cols(dy, c0s, bts, sc)
    for b in range(3):
        ref = sc[b] * dy[:, c0s[b]:c0s[b] + ncols[b]].float() @ bts[b].float().t()
        assert ((gl[b] - ref).norm() / ref.norm()) < 5e-3, b
    # dB of the 3 branches + dA of two dropout branches (keep bits) in one launch, accumulating into grads
    ps = [0.1, 0.0, 0.3]
    keys = [99, 0, 7]
    masks = torch.empty(3, M, K // 8, dtype=torch.uint8, device="cuda")
    As = [(torch.randn(16, K, device="cuda", generator=g) * 0.05).bfloat16() for _ in range(3)]
    xa = native_ext.lora_proj_m(x, As, [None] * 3, True, ps, keys, [1.0] * 3, masks)
    dB = [torch.full((n, 16), 0.25, device="cuda") for n in ncols]
    dA = [torch.zeros(16, K, device="cuda") for _ in range(3)]
    gs, xs, cs, ks, outs, ts, planes, pj = [], [], [], [], [], [], [], []
    for b in range(3):          # the dB jobs, then the dA jobs: consecutive jobs over x share its tiles
        gs.append(xa[b]), xs.append(dy), cs.append(c0s[b]), ks.append(ncols[b]), outs.append(dB[b])
        ts.append(True), planes.append(-1), pj.append(0.0)
    for b in range(3):
        gs.append(gl[b]), xs.append(x), cs.append(0), ks.append(K), outs.append(dA[b])
        ts.append(False), planes.append(b), pj.append(ps[b])
    native_ext.lora_acc_jobs(gs, xs, cs, ks, outs, ts, masks, planes, pj)
    for b in range(3):
        ref_b = 0.25 + dy[:, c0s[b]:c0s[b] + ncols[b]].float().t() @ xa[b]
        assert ((dB[b] - ref_b).norm() / ref_b.norm()) < 1e-2, ("dB", b)
        keep = _unpack(masks[b], K)
        ref_a = gl[b].t() @ (x.float() * keep / (1 - ps[b]))
        assert ((dA[b] - ref_a).norm() / ref_a.norm()) < 1e-2, ("dA", b)


@pytest.mark.parametrize("M,K,nbr", [(512, 1024, 3), (200, 512, 1), (2048, 4096, 4)])
def test_lora_dxc_matches_fp32(native_ext, M, K, nbr):
    g = torch.Generator(device="cuda").manual_seed(2)
    gs = [torch.randn(M, 16, device="cuda", generator=g) for _ in range(nbr)]
    As = [(torch.randn(16, K, device="cuda", generator=g) * 0.05).bfloat16() for _ in range(nbr)]
    ps = [0.05, 0.0, 0.2, 0.1][:nbr]
    masks = torch.randint(0, 256, (nbr, M, K // 8), dtype=torch.uint8, device="cuda", generator=g)
    ref = torch.zeros(M, K, device="cuda")
    for b in range(nbr):
        t = gs[b] @ As[b].float()
        if ps[b] > 0:
            t = t * _unpack(masks[b], K) / (1 - ps[b])
        ref += t
    for rb in (0, 1, 2, 4, 8):      # rows per wave (each form falls back to 1 where it would under-fill)
        c = native_ext.lora_dxc(gs, As, masks, ps, rb)
        assert ((c.float() - ref).norm() / ref.norm()) < 1e-2, rb


@pytest.mark.parametrize("nbr", [3, 1])
def test_fused_linear_multi_adapter_grads_match_fp32(native_ext, nbr):
    """One projection with 3 adapters (q|k|v: lora_dxc + the dX GEMM's C) or 1 (o: the masked term in the
    gemm4w dX prologue), dropout 0.1, against fp32 autograd with the kernels' own keep masks; B is large
    enough that the LoRA terms are a sizeable part of every gradient."""
    import llm_in_practise_amd.ops.linear as L
    g = torch.Generator(device="cuda").manual_seed(3)
    M, K = 512, 1024
    cols = [1024, 512, 512][:nbr] if nbr == 3 else [1024]
    N = sum(cols)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16().requires_grad_()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.03).bfloat16()
    p, s = 0.1, 2.0
    As = [(torch.randn(16, K, device="cuda", generator=g) * 0.05).requires_grad_() for _ in cols]
    Bs = [(torch.randn(n, 16, device="cuda", generator=g) * 0.3).requires_grad_() for n in cols]
    c0 = [0, 1024, 1536][:nbr] if nbr == 3 else [0]
    brs = [L.LoraBranch(a, b, s, p, c, c + n) for a, b, c, n in zip(As, Bs, c0, cols)]
    assert L._multi_ok(x, brs)
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    L.seed_dropout(7)
    y = L.fused_linear(x, w, None, brs, None, True)
    y.backward(dy)
    L.seed_dropout(7)
    keys = [L.next_dropout_key() for _ in cols]
    xr = x.detach().float().requires_grad_()
    Ar = [a.detach().clone().requires_grad_() for a in As]
    Br = [b.detach().clone().requires_grad_() for b in Bs]
    yr = xr @ w.float().t()
    parts = []
    for i, (c, n) in enumerate(zip(c0, cols)):
        keep = _keep(native_ext, M, K, p, keys[i])
        parts.append(s * ((xr * keep / (1 - p)) @ Ar[i].t()) @ Br[i].t())
    yr = yr + torch.cat(parts, 1)
    yr.backward(dy.float())
    assert ((y.float() - yr).norm() / yr.norm()) < 1e-2
    dx_base = dy.float() @ w.float()
    lora_k, lora_r = x.grad.float() - dx_base, xr.grad - dx_base
    assert ((lora_k - lora_r).norm() / lora_r.norm()) < 2e-2, "dx LoRA term"
    for i in range(nbr):
        assert ((As[i].grad - Ar[i].grad).norm() / Ar[i].grad.norm()) < 1e-2, ("dA", i)
        assert ((Bs[i].grad - Br[i].grad).norm() / Br[i].grad.norm()) < 1e-2, ("dB", i)


@pytest.mark.parametrize("quant,p", [(True, 0.1), (False, 0.1), (False, 0.0)])
def test_multi_adapter_path_matches_per_branch_kernels(native_ext, monkeypatch, quant, p):
    """q, k, v, o rank-16 adapters (3 on the fused q|k|v, 1 on o): the multi-adapter kernels give the loss
    and LoRA gradients of the per-adapter kernels (LIPA_LORA_MULTI=0), dropout included (same keys)."""
    import llm_in_practise_amd.ops.linear as L
    torch.manual_seed(0)
    ids = torch.randint(0, 1000, (2, 256), device="cuda")
    res = {}
    for mode in (False, True):
        monkeypatch.setattr(L, "_MULTI", mode)
        m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-small"), dtype=torch.bfloat16, device="cuda", seed=0)
        if quant:
            quantize_model_nf4(m)
        pm = get_peft_model(m, LoraConfig(r=16, lora_alpha=32, lora_dropout=p,
                                          target_modules=["q_proj", "k_proj", "v_proj", "o_proj"]))
        pm.fuse_projections()
        pm.train()
        for n, prm in pm.named_parameters():     # non-zero B so the dx / dA terms carry the masks
            if prm.requires_grad and "lora_B" in n:
                torch.nn.init.normal_(prm, std=0.02, generator=torch.Generator(device="cuda").manual_seed(hash(n) % 1000))
        L.seed_dropout(42)
        out = pm(input_ids=ids, labels=ids)
        out.loss.backward()
        res[mode] = (out.loss.item(), {n: prm.grad.float().clone() for n, prm in pm.named_parameters()
                                       if prm.requires_grad})
    (l0, g0), (l1, g1) = res[False], res[True]
    assert abs(l0 - l1) < 1e-3 * abs(l0)
    for n in g0:   # two bf16 paths 4 layers deep (the fp32 check is the op-level test above)
        err = (g0[n] - g1[n]).norm() / g0[n].norm().clamp(min=1e-12)
        assert err < 4e-2, (n, float(err))
