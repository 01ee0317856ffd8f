"""The non-reentrant activation checkpoint of the HIP path (ops/checkpoint.py _nonreentrant): use_reentrant=False
semantics without torch.utils.checkpoint's general machinery — same gradients as no checkpointing, inputs that do
not require grad, torch.autograd.grad, a retained graph backpropagated twice, the recompute mismatch guard, early
stop (an output no saved tensor needs is not recomputed)."""
import pytest
import torch

from llm_in_practise_amd.ops.checkpoint import _nonreentrant


def _mlp():
    torch.manual_seed(0)
    lin1, lin2 = torch.nn.Linear(16, 32), torch.nn.Linear(32, 8)

    def f(x, w):
        return lin2(torch.nn.functional.silu(lin1(x)) * w).sum(-1)
    return lin1, lin2, f


def test_same_gradients_as_plain_backward():
    lin1, lin2, f = _mlp()
    ps = [*lin1.parameters(), *lin2.parameters()]
    x = torch.randn(4, 16, requires_grad=True)
    w = torch.randn(32)
    _nonreentrant(f, (x, w)).sum().backward()
    g1 = [t.grad.clone() for t in [x, *ps]]
    for t in [x, *ps]:
        t.grad = None
    f(x, w).sum().backward()
    for a, t in zip(g1, [x, *ps]):
        assert torch.equal(a, t.grad)


def test_inputs_without_grad_autograd_grad_and_retained_graph():
    lin1, _, f = _mlp()
    w = torch.randn(32)
    y = _nonreentrant(f, (torch.randn(4, 16), w))            # no input requires grad: parameters still get grads
    y.sum().backward(retain_graph=True)
    a = lin1.weight.grad.clone()
    y.sum().backward()                                       # second backward through the retained graph
    assert torch.allclose(lin1.weight.grad, 2 * a)
    x = torch.randn(4, 16, requires_grad=True)
    g, = torch.autograd.grad(_nonreentrant(f, (x, w)).sum(), x)
    g2, = torch.autograd.grad(f(x, w).sum(), x)
    assert torch.equal(g, g2)


def test_recompute_taking_another_path_is_an_error():
    lin1, _, _ = _mlp()
    calls = [0]

    def f(x):
        calls[0] += 1
        h = lin1(x)
        return (h * h).sum() if calls[0] == 1 else h.sum()    # the recompute saves fewer tensors
    y = _nonreentrant(f, (torch.randn(2, 16),))
    with pytest.raises(RuntimeError, match="different code path"):
        y.backward()


class _Tail(torch.autograd.Function):
    """y = relu(x)·2 + x·w with the x·w term computed only when tail_skippable() says it is needed (the shape of the
    fused MLP: its own saved tensor first, then an output only later ops consume)."""
    computed = []

    @staticmethod
    def forward(ctx, x, w):
        from llm_in_practise_amd.ops.checkpoint import tail_skippable
        h = torch.relu(x)
        skip = tail_skippable(1)
        _Tail.computed.append(not skip)
        y = torch.empty_like(x) if skip else h * 2 + x * w
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * ((x > 0).to(g.dtype) * 2), None


def test_recompute_skips_an_output_no_saved_tensor_needs():
    """early stop: the op last to save anything leaves its output uncomputed in the recompute; gradients unchanged"""
    lin = torch.nn.Linear(8, 8)

    def layer(x, w):
        return _Tail.apply(lin(x), w)
    x = torch.randn(3, 8, requires_grad=True)
    w = torch.randn(8)
    _Tail.computed.clear()
    _nonreentrant(layer, (x, w)).sum().backward()
    assert _Tail.computed == [True, False]                    # forward computed y, the recompute skipped it
    g = [x.grad.clone(), lin.weight.grad.clone()]
    x.grad = lin.weight.grad = None
    layer(x, w).sum().backward()
    assert torch.equal(g[0], x.grad) and torch.equal(g[1], lin.weight.grad)


def test_recompute_keeps_an_output_a_later_saved_tensor_needs():
    """no early stop when an op after the tail point saves a tensor (its input would be the skipped output)"""
    lin = torch.nn.Linear(8, 8)

    def layer(x, w):
        y = _Tail.apply(lin(x), w)
        return (y * y).sum(-1)                                # y * y saves y
    x = torch.randn(3, 8, requires_grad=True)
    w = torch.randn(8)
    _Tail.computed.clear()
    _nonreentrant(layer, (x, w)).sum().backward()
    assert _Tail.computed == [True, True]
    g = x.grad.clone()
    x.grad = None
    layer(x, w).sum().backward()
    assert torch.equal(g, x.grad)
