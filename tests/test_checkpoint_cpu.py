"""The non-reentrant activation checkpoint of the HIP path (ops/checkpoint.py _nonreentrant): use_reentrant=False
semantics without torch.utils.checkpoint's general machinery — same gradients as no checkpointing, inputs that do
not require grad, torch.autograd.grad, a retained graph backpropagated twice, the recompute mismatch guard."""
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
