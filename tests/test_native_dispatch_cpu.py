"""ops/_native.py dispatch helpers: env_flag follows os.environ changes made at run time (monkeypatch.setenv, smoke()'s
LIPA_REFERENCE toggle), and fn_apply builds the same autograd graph as Function.apply."""
import torch

from llm_in_practise_amd.ops._native import env_flag, fn_apply, force_reference


def test_env_flag_tracks_runtime_changes(monkeypatch):
    monkeypatch.delenv("LIPA_REFERENCE", raising=False)
    assert not force_reference() and not env_flag("LIPA_REFERENCE")
    monkeypatch.setenv("LIPA_REFERENCE", "1")
    assert force_reference()
    monkeypatch.setenv("LIPA_REFERENCE", "0")
    assert not force_reference()


class _Scale(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, k):
        ctx.save_for_backward(w)
        ctx.k = k
        return x * w * k

    @staticmethod
    def backward(ctx, g):
        (w,) = ctx.saved_tensors
        return g * w * ctx.k, None, None


def test_fn_apply_matches_function_apply():
    x = torch.randn(5, requires_grad=True)
    w = torch.randn(5)
    y1 = _Scale.apply(x, w, 3.0)
    g1, = torch.autograd.grad(y1.sum(), x)
    y2 = fn_apply(_Scale, x, w, 3.0)
    g2, = torch.autograd.grad(y2.sum(), x)
    assert torch.equal(y1, y2) and torch.equal(g1, g2)
    assert type(y2.grad_fn).__name__ == type(y1.grad_fn).__name__
    with torch.no_grad():
        assert fn_apply(_Scale, x, w, 2.0).grad_fn is None
