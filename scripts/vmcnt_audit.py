#!/usr/bin/env python3
"""Structural check of counted vector-memory waits in the gfx950 ISA of the LDS-DMA kernels.

``s_waitcnt vmcnt(N)`` with N > 0 waits until at most N of the wave's vector-memory operations are
outstanding.  The kernels here stage tiles with LDS-DMA (``buffer_load_dwordx4 … lds``) and count those
DMAs with explicit waits.  A counted wait is a correct guard for a REGISTER load only if the load cannot
still be in flight when the count is reached, i.e. only if vector-memory operations of different kinds retire
in issue order AND the compiler never copies the (asm) destination registers before the wait — neither is
guaranteed.  The round-5 dK/dV race (profiles/r5/zero3_dkv_race.txt) was exactly that: lse / delta register
loads issued beside the next tile's DMAs and guarded by ``vmcnt(8)``; under contention a stale value fed P / dS.

Rule checked here, per kernel, by a linear scan of the device assembly (``hipcc -S --offload-arch=gfx950``):
while any LDS-DMA is outstanding (since the last full drain ``vmcnt(0)``), a counted wait ``vmcnt(N > 0)`` must
not be the wait that covers a register-destination load — every operation older than the N youngest must be
an LDS-DMA or a store.  Register loads beside DMAs are drained by ``vmcnt(0)`` instead.

    python scripts/vmcnt_audit.py llm_in_practise_amd/csrc/kernels/attention.hip ...
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
KDIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "llm_in_practise_amd", "csrc",
                    "kernels")
_VMEM = re.compile(r"^\s*(global|buffer|flat)_(load|store|atomic)\w*")
_WAIT = re.compile(r"^\s*s_waitcnt\b(.*)")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")


def device_asm(src: str, arch: str = "gfx950", cache_dir: str | None = None) -> str:
    """Device-only assembly of one HIP source with the extension's kernel flags (csrc/build.py); cached under
    ``cache_dir`` by the contents of the source and of the kernel headers."""
    import glob
    import hashlib
    h = hashlib.sha1(arch.encode())
    for p in [src] + sorted(glob.glob(os.path.join(KDIR, "*.h"))):
        with open(p, "rb") as f:
            h.update(f.read())
    cached = os.path.join(cache_dir, f"{os.path.basename(src)}.{h.hexdigest()[:16]}.s") if cache_dir else None
    if cached and os.path.exists(cached):
        with open(cached) as f:
            return f.read()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        cmd = [os.path.join(ROCM, "bin", "hipcc"), "-x", "hip", "-O3", "-std=c++17", f"--offload-arch={arch}",
               "--offload-device-only", "-S", "-munsafe-fp-atomics", "-ffp-contract=fast", f"-I{KDIR}", src, "-o", out]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc -S failed for {src}:\n{r.stderr[-4000:]}")
        with open(out) as f:
            text = f.read()
    if cached:
        os.makedirs(cache_dir, exist_ok=True)
        with open(cached + ".tmp", "w") as f:
            f.write(text)
        os.replace(cached + ".tmp", cached)
    return text


def _kind(line: str) -> str:
    op = _VMEM.match(line).group(0).strip()
    if " lds" in line or op.startswith(("global_load_lds", "buffer_load_lds")):
        return "dma"
    if "_store" in op or ("_atomic" in op and " glc" not in line and " sc0" not in line):
        return "store"
    return "load"


def audit(asm: str) -> tuple[list[str], dict]:
    """Return (violations, stats) over every function of the assembly text."""
    violations: list[str] = []
    stats = {"functions": 0, "counted_waits": 0, "counted_waits_beside_dma": 0, "dma_ops": 0}
    fn = None
    window: list[tuple[str, int]] = []
    for no, raw in enumerate(asm.splitlines(), 1):
        line = raw.split(";")[0].rstrip() if not raw.lstrip().startswith(";") else ""
        m = re.match(r"^([A-Za-z_][\w.$]*):", raw)
        if m and not m.group(1).startswith((".L", "$")):
            fn = m.group(1)
            window = []
            stats["functions"] += 1
            continue
        if not line:
            continue
        if _VMEM.match(line):
            k = _kind(line)
            window.append((k, no))
            stats["dma_ops"] += k == "dma"
            continue
        w = _WAIT.match(line)
        if not w:
            continue
        mv = _VMCNT.search(w.group(1))
        if mv is None:
            nums = re.findall(r"0x[0-9a-fA-F]+|\b\d+\b", w.group(1))
            if not nums:
                continue
            imm = int(nums[0], 0)                     # raw gfx9 encoding: vmcnt = [3:0] | [15:14] << 4
            n = (imm & 0xF) | (((imm >> 14) & 3) << 4)
        else:
            n = int(mv.group(1))
        if n == 0:
            window = []
            continue
        stats["counted_waits"] += 1
        covered, window = window[:-n] if len(window) > n else [], window[-n:]
        if any(k == "dma" for k, _ in covered + window):
            stats["counted_waits_beside_dma"] += 1
            bad = [ln for k, ln in covered if k == "load"]
            if bad:
                violations.append(f"{fn}: line {no} `{line.strip()}` covers register load(s) at line(s) "
                                  f"{bad[:4]} while LDS-DMAs are outstanding")
    return violations, stats


# every source whose kernels issue LDS-DMA (buffer_load … lds)
DMA_SOURCES = ("attention.hip", "gemm4w.hip", "gemm4w_lora.hip", "gemm4w_mlp.hip")


def audit_sources(srcs=None, cache_dir: str | None = None, jobs: int = 4) -> dict:
    """{source: (violations, stats)} for the given (default: DMA_SOURCES) kernel sources, compiled in parallel."""
    import concurrent.futures as cf
    srcs = srcs or [os.path.join(KDIR, f) for f in DMA_SOURCES]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        asms = list(ex.map(lambda s: device_asm(s, cache_dir=cache_dir), srcs))
    return {s: audit(a) for s, a in zip(srcs, asms)}


def main(argv):
    rc = 0
    for s, (v, st) in audit_sources(argv or None).items():
        print(f"{os.path.basename(s)}: {st}")
        for x in v:
            print("  VIOLATION", x)
        rc |= bool(v)
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
