"""Benchmark harness (SURVEY.md §7.1 ``bench/``).

* :mod:`.scaling` — run the headline ``bench.py`` at 1 / 2 / 4 / 8 GPUs of one node (each N as
  its own ``torch.distributed.run`` job over RCCL) and report the scaling curve: whole-node
  tokens/s, per-GPU tokens/s and weak-scaling efficiency against N = 1
  (BASELINE.md "report padded and non-pad tokens/s for 1, 2, 4 and 8 GPUs as a scaling curve").
* ``scripts/bench_serve.py`` — serving (TTFT / ITL / throughput at the reference's concurrency
  levels), ``scripts/bench_gemm4w.py`` / ``bench_w4.py`` / ``bench_attn.py`` / ``bench_decode.py`` — kernel A/Bs.
"""
