"""CPU tests: fused optimizer references, schedulers, host C++ runtime (CPU Adam, loader)."""
import math

import torch

from llm_in_practise_amd.optim.adamw import AdamW, AdamW8bit, LRScheduler, build_optimizer


def test_adamw_reference_matches_torch():
    torch.manual_seed(0)
    p1 = torch.nn.Parameter(torch.randn(1000))
    p2 = torch.nn.Parameter(p1.detach().clone())
    o1 = AdamW([p1], lr=1e-2, weight_decay=0.1)
    o2 = torch.optim.AdamW([p2], lr=1e-2, weight_decay=0.1)
    for _ in range(5):
        g = torch.randn(1000)
        p1.grad.copy_(g)
        p2.grad = g.clone()
        o1.step()
        o2.step()
    assert torch.allclose(p1.detach(), p2.detach(), atol=1e-6)


def test_flat_grads_accumulate_in_place():
    lin = torch.nn.Linear(8, 4)
    opt = AdamW(lin.parameters(), lr=1e-3)
    x = torch.randn(3, 8)
    lin(x).sum().backward()
    g1 = opt.grad_buffer.clone()
    lin(x).sum().backward()
    assert torch.allclose(opt.grad_buffer, 2 * g1)
    assert lin.weight.grad.data_ptr() >= opt.grad_buffer.data_ptr()
    opt.zero_grad()
    assert opt.grad_buffer.abs().sum() == 0


def test_clip_coefficient():
    p = torch.nn.Parameter(torch.zeros(100))
    opt = AdamW([p], lr=1.0)
    p.grad.fill_(1.0)
    n = opt.clip_grad_norm_(1.0)
    assert abs(n.item() - 10.0) < 1e-5 and abs(opt.norm_out[1].item() - 0.1) < 1e-6


def test_adamw8bit_reference_tracks_fp32():
    torch.manual_seed(0)
    p1 = torch.nn.Parameter(torch.randn(2048))
    p2 = torch.nn.Parameter(p1.detach().clone())
    o1, o2 = AdamW8bit([p1], lr=1e-3), AdamW([p2], lr=1e-3, weight_decay=0.0)
    for _ in range(10):
        g = torch.randn(2048)
        p1.grad.copy_(g)
        p2.grad.copy_(g)
        o1.step()
        o2.step()
    assert (p1 - p2).norm() / (p2.detach() - p1.detach() + p2.detach()).norm() < 5e-3


def test_state_dict_roundtrip():
    p = torch.nn.Parameter(torch.randn(64))
    o = build_optimizer("adamw_torch", [p], 1e-3)
    p.grad.normal_()
    o.step()
    sd = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in o.state_dict().items()}
    sd["state"] = {k: v.clone() for k, v in sd["state"].items()}
    p2 = torch.nn.Parameter(torch.zeros(64))
    o2 = build_optimizer("adamw_torch", [p2], 1e-3)
    o2.load_state_dict(sd)
    assert torch.allclose(p2.detach(), p.detach()) and o2.step_count == 1


def test_schedulers():
    p = torch.nn.Parameter(torch.zeros(4))
    o = AdamW([p], lr=1.0)
    s = LRScheduler(o, "linear", 1.0, total_steps=10)
    lrs = [s.get_last_lr()[0]] + [(s.step(), s.get_last_lr()[0])[1] for _ in range(10)]
    assert lrs[0] == 1.0 and abs(lrs[5] - 0.5) < 1e-9 and lrs[-1] == 0.0
    c = LRScheduler(o, "cosine", 1.0, total_steps=10, warmup_steps=2)
    assert abs(c.lr_at(0) - 0.5) < 1e-9 and abs(c.lr_at(6) - 0.5) < 1e-9
    w = LRScheduler(o, "warmup_lr", 3e-4, total_steps=1000, warmup_steps=100)
    assert w.lr_at(0) == 0.0 and abs(w.lr_at(99) - 3e-4) < 1e-12 and w.lr_at(500) == 3e-4
    st = LRScheduler(o, "step", 1.0, total_steps=10, gamma=0.95)
    assert abs(st.lr_at(2) - 0.95 ** 2) < 1e-12


def test_cpu_adam_native_matches_reference():
    from llm_in_practise_amd.ops._native import cpu_native
    from llm_in_practise_amd.ops.reference import adamw_step
    C = cpu_native()
    torch.manual_seed(0)
    p = torch.randn(10_000)
    g = torch.randn(10_000)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    p16 = torch.empty(10_000, dtype=torch.bfloat16)
    for step in range(1, 4):
        C.adamw_step(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, 1.0, p16)
        adamw_step(p2, g, m2, v2, step, 1e-3, 0.9, 0.999, 1e-8, 0.01)
    assert torch.allclose(p, p2, atol=1e-6)
    assert torch.allclose(p16.float(), p, atol=1e-2)
    assert math.isclose(C.sum_squares(g), g.double().pow(2).sum().item(), rel_tol=1e-9)


def test_token_block_loader_sharding_and_resume():
    from llm_in_practise_amd.ops._native import cpu_native
    C = cpu_native()
    toks = torch.arange(33 * 64)                                    # 64 blocks of 32+1
    seen = []
    for r in range(2):
        L = C.TokenBlockLoader(toks, 32, 4, r, 2, 7, True, 2, False)
        assert L.steps_per_epoch == 8
        for _ in range(L.steps_per_epoch):
            x, y = L.next()
            assert torch.equal(y, x + 1)
            seen += (x[:, 0] // 33).tolist()
    assert sorted(seen) == list(range(64))                           # ranks partition the epoch
    L = C.TokenBlockLoader(toks, 32, 4, 0, 1, 7, True, 2, False)
    a = [L.next()[0] for _ in range(5)]
    L2 = C.TokenBlockLoader(toks, 32, 4, 0, 1, 7, True, 2, False)
    L2.start_epoch(0, 3)
    assert torch.equal(L2.next()[0], a[3])                            # exact resume


def _two_groups(ps):
    """decay / no-decay split with different lrs (temp/ddp_gpt_wikitext2.py:337-344 shape)"""
    return [{"params": [ps[0]], "weight_decay": 0.1, "lr": 1e-2}, {"params": [ps[1], ps[2]], "weight_decay": 0.0, "lr": 3e-3}]


def test_adamw_param_groups_match_torch():
    torch.manual_seed(0)
    shapes = [(33, 7), (7,), (300,)]
    a = [torch.nn.Parameter(torch.randn(s)) for s in shapes]
    b = [torch.nn.Parameter(t.detach().clone()) for t in a]
    o1 = AdamW(_two_groups(a), lr=5e-4)
    o2 = torch.optim.AdamW(_two_groups(b), lr=5e-4)
    assert len(o1.param_groups) == 2 and o1.param_groups[1]["lr"] == 3e-3
    for _ in range(4):
        for p1, p2 in zip(a, b):
            g = torch.randn(p1.shape)
            p1.grad.copy_(g)
            p2.grad = g.clone()
        o1.step()
        o2.step()
    for p1, p2 in zip(a, b):
        assert torch.allclose(p1.detach(), p2.detach(), atol=1e-6)


def test_adamw8bit_param_groups_update_every_group():
    torch.manual_seed(0)
    a = [torch.nn.Parameter(torch.randn(s)) for s in [(300,), (5,), (700,)]]
    b = [torch.nn.Parameter(t.detach().clone()) for t in a]
    o1 = AdamW8bit(_two_groups(a))
    o2 = AdamW(_two_groups(b))
    for _ in range(6):
        for p1, p2 in zip(a, b):
            g = torch.randn(p1.shape)
            p1.grad.copy_(g)
            p2.grad.copy_(g)
        o1.step()
        o2.step()
    for p1, p2, p0 in zip(a, b, [torch.randn(1)] * 3):
        assert (p1 - p2).norm() / (p2.detach()).norm() < 5e-3


def test_scheduler_scales_each_group():
    ps = [torch.nn.Parameter(torch.randn(4)) for _ in range(3)]
    o = AdamW(_two_groups(ps), lr=1e-2)
    sch = LRScheduler(o, "linear", 1e-2, total_steps=10)
    sch.step()
    lrs = sch.get_last_lr()
    assert abs(lrs[0] - 0.9e-2) < 1e-12 and abs(lrs[1] - 0.9 * 3e-3) < 1e-12
