"""Tensor-parallel inference (vLLM ``--tensor-parallel-size`` parity) on CPU with gloo.

Oracle: the unsharded model in the same process.  TP=2 (and TP=4 for the head split) must give
the same logits, the same greedy generation, and must keep a LoRA adapter's contribution
(column-parallel lora_B rows / row-parallel lora_A columns).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(arch, lora, layers=2):
    cfg = qwen3_config(arch, num_attention_heads=4, num_key_value_heads=4 if arch == "qwen2-tiny" else 2,
                       num_hidden_layers=layers)
    m = Qwen3ForCausalLM.from_config(cfg, dtype=torch.float32, device="cpu", seed=3)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith(".bias"):
                p.normal_(0, 0.05)
    if lora:
        from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model
        m = get_peft_model(m, LoraConfig(r=4, lora_alpha=8, lora_dropout=0.0,
                                         target_modules=["q_proj", "v_proj", "o_proj", "down_proj"]))
        with torch.no_grad():
            for n, p in m.named_parameters():
                if "lora_B" in n:
                    p.normal_(0, 0.05)
    m.eval()
    return m


def _worker(rank, world, port, arch, lora, q, pp=1, layers=2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from llm_in_practise_amd.parallel.pipeline_parallel import apply_pipeline_parallel, make_tp_pp_groups
        from llm_in_practise_amd.parallel.tensor_parallel import apply_tensor_parallel
        torch.manual_seed(0)
        ids = torch.randint(0, 512, (2, 12))
        ref_model = _model(arch, lora, layers)
        with torch.no_grad():
            ref = ref_model(ids).logits
            ref_gen = ref_model.generate(ids, max_new_tokens=6, do_sample=False) if not lora else None
        tpg, ppg = make_tp_pp_groups(world // pp, pp)
        tp_model = _model(arch, lora, layers)
        if ppg is not None:
            apply_pipeline_parallel(tp_model, ppg)
            n_local = len(next(m for m in tp_model.modules() if hasattr(m, "embed_tokens")).layers)
            assert n_local < layers
        if tpg is not None:
            apply_tensor_parallel(tp_model, tpg)
        with torch.no_grad():
            out = tp_model(ids).logits
            gen = tp_model.generate(ids, max_new_tokens=6, do_sample=False) if not lora else None
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        same_gen = True if ref_gen is None else bool(torch.equal(gen, ref_gen))
        q.put((rank, err, same_gen))
    finally:
        torch.distributed.destroy_process_group()


def _run(world, arch, lora, pp=1, layers=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, arch, lora, q, pp, layers)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,arch,lora", [(2, "qwen3-tiny", False), (2, "qwen2-tiny", True),
                                             (4, "qwen2-tiny", False)])
def test_tp_matches_single_process(world, arch, lora):
    for rank, err, same_gen in _run(world, arch, lora):
        assert err < 1e-5, (rank, err)
        assert same_gen, rank


@pytest.mark.parametrize("world,pp,arch,lora,layers", [(2, 2, "qwen3-tiny", False, 3), (2, 2, "qwen2-tiny", True, 2),
                                                       (4, 2, "qwen3-tiny", False, 3)])
def test_pp_matches_single_process(world, pp, arch, lora, layers):
    """Pipeline parallel: stages of 2+1 layers (uneven split), with a LoRA adapter,
    and TP=2 x PP=2 over 4 ranks, all equal to the unsharded model."""
    for rank, err, same_gen in _run(world, arch, lora, pp, layers):
        assert err < 1e-5, (rank, err)
        assert same_gen, rank


def _engine_worker(rank, world, port, q, pp=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from llm_in_practise_amd.infer.engine import SamplingParams, ServingEngine
        from llm_in_practise_amd.parallel.tensor_parallel import apply_tensor_parallel
        from llm_in_practise_amd.train.data import ByteTokenizer
        tok = ByteTokenizer()
        tok.eos_token_id = 10
        cfg = qwen3_config("qwen3-tiny", vocab_size=256)
        single = None
        if rank == 0:       # oracle: the unsharded model in an ordinary engine
            m1 = Qwen3ForCausalLM.from_config(cfg, dtype=torch.float32, seed=0).eval()
            e1 = ServingEngine(m1, tok, max_batch=4)
            p = SamplingParams(max_tokens=8, temperature=0.0)
            single = [e1.complete(s, p)["text"] for s in ("abc", "hello", "tensor parallel")]
            e1.shutdown()
        m = Qwen3ForCausalLM.from_config(cfg, dtype=torch.float32, seed=0).eval()
        if pp > 1:
            from llm_in_practise_amd.parallel.pipeline_parallel import apply_pipeline_parallel
            m = apply_pipeline_parallel(m)
        else:
            m = apply_tensor_parallel(m)
        eng = ServingEngine(m, tok, max_batch=4, tp_group=torch.distributed.group.WORLD)
        if rank == 0:
            p = SamplingParams(max_tokens=8, temperature=0.0)
            reqs = [eng.submit(s, p) for s in ("abc", "hello", "tensor parallel")]
            outs = []
            for r in reqs:
                while True:
                    kind, val = r.out.get(timeout=120)
                    if kind == "final":
                        outs.append(val["text"])
                        break
            eng.shutdown()
            eng._worker.join(timeout=60)
            q.put((rank, outs == single, outs, single))
        else:
            eng.follower_loop()
            q.put((rank, True, None, None))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("pp", [1, 2])
def test_tp_serving_engine_spmd(pp):
    """vLLM-style TP / PP serving: rank 0 owns the queue, followers replay its iterations."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_engine_worker, args=(r, 2, port, q, pp)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, outs, single in res:
        assert ok, (rank, outs, single)
