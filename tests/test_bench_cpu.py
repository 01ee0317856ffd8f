"""bench.py contract on CPU (gloo, 2 ranks): one JSON line from rank 0 with the driver's fields,
whole-job tokens/s, weak scaling, for the DDP and ZeRO-3 strategies and both GA executions."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_self_launches_n_ranks():
    """`python bench.py --gpus 2` (no launcher env) must start 2 ranks itself, not silently run 1."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--model", "qwen3-tiny", "--seq-len", "64"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["dist_world_size"] == 2
    assert d["config"]["parallelism"] == "dp2"


@pytest.mark.parametrize("extra", [[], ["--ga-fusion", "0"], ["--strategy", "zero3"]])
def test_bench_json_contract_two_ranks(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--model", "qwen3-tiny", "--seq-len", "64", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 only
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["higher_is_better"] is True and d["value"] > 0 and d["ms_per_step"] > 0
    tokens = 2 * 64 * 2 * 2 * 2                  # micro 2 x seq 64 x GA 2 x world 2 x steps 2
    assert abs(d["value"] - tokens / (d["ms_per_step"] * 2 / 1000)) / d["value"] < 0.02
    assert d["config"]["global_batch"] == 8
    assert d["config"]["parallelism"] == ("zero3-dp2" if "zero3" in extra else "dp2")
    # kernel provenance: GEMM launches per step by form (CPU: every GEMM is the torch fallback)
    c = d["config"]
    assert c["gemm_backend"] == "torch-cpu" and c["gemm_launches_per_step"]["library"] > 0
    assert "nf4_expansions_per_step" in c and c["gemm_launches_per_step"].get("gemm4w", 0) == 0
    # host issue time of one step onto an idle device (a measure of launch-boundness; CPU: the whole step)
    assert d["host_launch_ms"] is None or d["host_launch_ms"] > 0
    _check_comm(d["comm"], "all_gather" if "zero3" in extra else "all_reduce")
    if "zero3" not in extra:       # the DDP headline carries BASELINE #4 (ZeRO-3) as a sub-record at world > 1
        _check_zero3(d["zero3"], 2)


def _check_comm(c, kind):
    """the per-step collective record of a multi-rank bench line (parallel/dist.py CommStats)"""
    assert c["steps"] >= 1 and kind in c, c
    assert c[kind]["calls_per_step"] > 0 and c[kind]["mbytes_per_step"] > 0
    assert c[kind]["exposed_ms_per_step"] >= 0 and "overlap_fraction" in c and "exposed_ms_per_step" in c


def _check_zero3(z, world):
    assert "error" not in z, z
    for k in ("model", "value", "unit", "ms_per_step", "steps", "warmup", "n_gpus", "parallelism", "ds_config",
              "optimizer", "global_batch", "dist_backend", "comm"):
        assert k in z, k
    assert z["n_gpus"] == world and z["parallelism"] == f"zero3-dp{world}" and z["value"] > 0
    assert z["optimizer"] == "zero3-paged_adamw_8bit" and z["ds_config"].endswith("ds_zero3_config.json")
    _check_comm(z["comm"], "reduce_scatter")
    _check_comm(z["comm"], "all_gather")


def test_bench_zero3_subrecord_four_ranks():
    """world 4 (gloo): the headline DDP line carries the zero3 sub-record and both comm records"""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "4", "--steps", "1", "--warmup", "1", "--model", "qwen3-tiny", "--seq-len", "64",
           "--faithful-steps", "0", "--selective-steps", "0", "--zero3-steps", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    _check_comm(d["comm"], "all_reduce")
    _check_zero3(d["zero3"], 4)


def test_scaling_harness_runs_each_world_size(tmp_path):
    """bench/scaling.py: one bench.py job per N (gloo on CPU), efficiency vs N = 1."""
    out = tmp_path / "scale.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, "-m", "llm_in_practise_amd.bench.scaling", "--gpus", "1", "2", "--steps", "1",
                        "--warmup", "1", "--out", str(out), "--model", "qwen3-tiny", "--seq-len", "64"],
                       capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert [t["n_gpus"] for t in d["table"]] == [1, 2]
    assert d["table"][0]["weak_scaling_efficiency"] == 1.0 and d["table"][1]["weak_scaling_efficiency"] > 0


def test_awq_infer_bench_tiny(tmp_path):
    """BASELINE #5 harness: merged LoRA -> AWQ int4, decode/prefill/serve on both, quality vs bf16."""
    out = tmp_path / "awq.json"
    r = subprocess.run([sys.executable, "-m", "llm_in_practise_amd.bench.awq_infer", "--model", "qwen3-tiny",
                        "--batches", "1", "4", "--steps", "2", "--prefill", "2", "64", "--ppl-prompts", "2",
                        "--ppl-new", "8", "--calib", "2", "--calib-len", "64", "--group-size", "32",
                        "--serve-requests", "4", "--serve-tokens", "8", "--max-len", "256", "--ctx", "32",
                        "--out", str(out)], capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["int4"]["weight_bytes"] < 0.35 * d["bf16"]["weight_bytes"]
    assert d["int4"]["kl_vs_bf16"] < 0.05 and d["int4"]["top1_agree_vs_bf16"] > 0.5
    assert d["int4"]["serve"]["output_tok_per_s"] > 0
    assert [x["batch"] for x in d["int4"]["decode"]] == [1, 4]


def _bench_with_fault(world, fault, extra=(), hang_s=None, timeout=600):
    env = dict(os.environ, OMP_NUM_THREADS="1", LIPA_BENCH_FAULT=fault)
    if hang_s is not None:
        env["FAULT_HANG_S"] = str(hang_s)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "1", "--warmup", "1", "--model", "qwen3-tiny", "--seq-len", "64",
           "--host-steps", "1", "--zero3-steps", "2", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["n_gpus"] == world   # the headline survived
    _check_comm(d["comm"], "all_reduce")
    return d, r.stderr


@pytest.mark.parametrize("world,fault", [(2, "zero3=1:0:raise"), (4, "zero3=*:1:raise"), (4, "zero3=2:0:raise")])
def test_bench_headline_survives_zero3_failure(world, fault):
    """a failure inside the ZeRO-3 sub-record (one rank or all) is recorded as zero3.error; the headline line is
    printed and the job exits 0 (bench.py sub())"""
    d, _ = _bench_with_fault(world, fault, ["--faithful-steps", "0", "--selective-steps", "0"])
    assert "error" in d["zero3"], d["zero3"]


def test_bench_headline_survives_zero3_hang():
    """a rank that hangs inside the ZeRO-3 sub-record: every rank's watchdog ends the sub-record after its budget,
    rank 0 prints the headline with the watchdog's error"""
    d, err = _bench_with_fault(2, "zero3=1:0:hang", ["--faithful-steps", "0", "--selective-steps", "0",
                                                     "--subrecord-budget-s", "15"], hang_s=300)
    assert d["zero3"]["error"].startswith("watchdog"), d["zero3"]
    assert "[watchdog] rank 0" in err


def test_bench_faithful_failure_skips_later_subrecords():
    """a failure in the faithful sub-record at world 2: recorded; the later sub-records are skipped on that rank
    (its peers may still be inside a collective) and the headline is printed"""
    d, _ = _bench_with_fault(2, "faithful=*:0:raise", ["--faithful-steps", "2", "--selective-steps", "1"])
    assert "error" in d["faithful"]
    assert "skipped" in d["selective_ckpt"] and "skipped" in d["zero3"]
    assert d["host_launch_ms"] is not None and d["host_launch_ms"] > 0
