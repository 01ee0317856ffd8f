"""Scaling curve of the headline benchmark: ``python -m llm_in_practise_amd.bench.scaling``.

    python -m llm_in_practise_amd.bench.scaling --gpus 1 2 4 8 --steps 20 --warmup 5 [bench.py args...]

Each N runs ``bench.py --gpus N`` (which starts N ranks under ``torch.distributed.run`` itself)
in a fresh process, one after another; the JSON line of every run is parsed and the table
printed (and written with ``--out``).  Weak scaling: per-GPU work is fixed, so ideal whole-node
tokens/s is N × the 1-GPU value; efficiency = value_N / (N · value_1).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_one(n: int, steps: int, warmup: int, extra: list[str], timeout: int = 3600) -> dict:
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(steps),
           "--warmup", str(warmup), *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        raise RuntimeError(f"bench.py --gpus {n} failed ({r.returncode}):\n{r.stderr[-2000:]}")
    return json.loads(lines[-1])


def table(rows: list[dict]) -> list[dict]:
    base = next((r for r in rows if r["n_gpus"] == 1), None)
    out = []
    for r in rows:
        n = r["n_gpus"]
        eff = (r["value"] / (n * base["value"])) if base else None
        out.append({"n_gpus": n, "tokens_per_s": r["value"], "tokens_per_s_per_gpu": round(r["value"] / n, 1),
                    "ms_per_step": r["ms_per_step"], "weak_scaling_efficiency": round(eff, 3) if eff else None,
                    "nonpad_tokens_per_s": r["config"].get("tokens_per_s_nonpad")})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default=None)
    a, extra = ap.parse_known_args(argv)
    rows = [run_one(n, a.steps, a.warmup, extra) for n in a.gpus]
    t = table(rows)
    print(f"{'GPUs':>5} {'tok/s (node)':>14} {'tok/s/GPU':>11} {'ms/step':>9} {'weak eff':>9}")
    for r in t:
        eff = "-" if r["weak_scaling_efficiency"] is None else f"{r['weak_scaling_efficiency']:.3f}"
        print(f"{r['n_gpus']:>5} {r['tokens_per_s']:>14,.0f} {r['tokens_per_s_per_gpu']:>11,.0f} "
              f"{r['ms_per_step']:>9.2f} {eff:>9}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"runs": rows, "table": t}, f, indent=2)
    return 0


if __name__ == "__main__":
    sys.exit(main())
