"""MoE routing / dispatch ops (K14): CPU path against a plain index_add formulation, HIP
kernels against the fp32 torch reference (values and gradients)."""
import pytest
import torch
import torch.nn.functional as F

from llm_in_practise_amd.ops.moe import moe_combine, moe_dispatch, moe_gather, moe_route


def _plain_moe(x, logits, k, experts, mode):
    """The reference's sparse formulation: top-k, per-expert gather, index_add_."""
    if mode == "topk_softmax":
        top, idx = logits.float().topk(k, -1)
        w = F.softmax(top, -1)
    else:
        w, idx = F.softmax(logits.float(), -1).topk(k, -1)
    out = torch.zeros_like(x)
    for j in range(k):
        for e, f in enumerate(experts):
            sel = (idx[:, j] == e).nonzero().squeeze(-1)
            if sel.numel():
                out.index_add_(0, sel, f(x[sel]) * w[sel, j:j + 1].to(x.dtype))
    return out


def _ours(x, logits, k, experts, mode, base=None):
    w, idx = moe_route(logits, k, mode)
    d = moe_dispatch(idx, len(experts))
    xs = moe_gather(x, d)
    ys, s = [], 0
    for e, c in enumerate(d.counts()):
        if c:
            ys.append(experts[e](xs[s:s + c]))
        s += c
    return moe_combine(torch.cat(ys, 0), d, w, base)


@pytest.mark.parametrize("mode", ["topk_softmax", "softmax_topk"])
def test_moe_dispatch_cpu_matches_index_add(mode):
    torch.manual_seed(0)
    T, H, E, k = 37, 16, 6, 2
    x = torch.randn(T, H, requires_grad=True)
    logits = torch.randn(T, E, requires_grad=True)
    mats = [torch.randn(H, H) * 0.3 for _ in range(E)]
    experts = [lambda z, m=m: torch.tanh(z @ m) for m in mats]
    ref = _plain_moe(x, logits, k, experts, mode)
    ours = _ours(x, logits, k, experts, mode)
    torch.testing.assert_close(ours, ref, rtol=1e-5, atol=1e-5)
    g = torch.randn_like(ref)
    gx_r, gl_r = torch.autograd.grad(ref, (x, logits), g)
    gx_o, gl_o = torch.autograd.grad(ours, (x, logits), g)
    torch.testing.assert_close(gx_o, gx_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gl_o, gl_r, rtol=1e-5, atol=1e-5)


def test_dispatch_is_stable_and_segmented():
    idx = torch.tensor([[2, 0], [0, 1], [2, 1], [0, 2]])
    d = moe_dispatch(idx, 4)
    assert d.counts() == [3, 2, 3, 0]
    flat = idx.reshape(-1)
    perm = d.perm.long()
    assert torch.equal(flat[perm], torch.sort(flat, stable=True).values)
    assert perm.tolist() == [1, 2, 6, 3, 5, 0, 4, 7]     # token order kept inside each expert
    assert torch.equal(perm[d.pos_of.long()], torch.arange(8))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode", ["topk_softmax", "softmax_topk"])
def test_moe_kernels_match_reference(dtype, mode):
    from llm_in_practise_amd.ops._native import native
    native()
    torch.manual_seed(0)
    dev = "cuda"
    T, H, E, k = 1000, 256, 8, 2
    x = torch.randn(T, H, device=dev, dtype=dtype, requires_grad=True)
    logits = torch.randn(T, E, device=dev, dtype=dtype, requires_grad=True)
    base = torch.randn(T, H, device=dev, dtype=dtype, requires_grad=True)
    mats = [torch.randn(H, H, device=dev, dtype=dtype) * 0.05 for _ in range(E)]
    experts = [lambda z, m=m: torch.tanh(z @ m) for m in mats]
    ours = _ours(x, logits, k, experts, mode, base)
    # fp32 reference on CPU
    xr, lr, br = (t.detach().float().cpu().requires_grad_(True) for t in (x, logits, base))
    mats_r = [m.float().cpu() for m in mats]
    ref = _plain_moe(xr, lr, k, [lambda z, m=m: torch.tanh(z @ m) for m in mats_r], mode) + br
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ours.float().cpu(), ref, **tol)
    g = torch.randn(T, H, device=dev, dtype=dtype)
    gx, gl, gb = torch.autograd.grad(ours, (x, logits, base), g)
    gxr, glr, gbr = torch.autograd.grad(ref, (xr, lr, br), g.float().cpu())
    torch.testing.assert_close(gx.float().cpu(), gxr, **tol)
    torch.testing.assert_close(gl.float().cpu(), glr, **tol)
    torch.testing.assert_close(gb.float().cpu(), gbr, **tol)


@pytest.mark.gpu
def test_moe_permute_kernel_many_pairs():
    from llm_in_practise_amd.ops._native import native
    torch.manual_seed(1)
    idx = torch.randint(0, 64, (5000, 6), device="cuda")
    d = moe_dispatch(idx, 64)
    flat = idx.reshape(-1).cpu()
    perm = d.perm.long().cpu()
    assert torch.equal(perm, torch.argsort(flat, stable=True))
    assert torch.equal(d.offsets.cpu()[1:] - d.offsets.cpu()[:-1], torch.bincount(flat, minlength=64).int())
    assert native() is not None
