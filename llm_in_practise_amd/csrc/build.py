"""Native build driver — hipcc / g++ directly, no torch hipify pass.

``torch.utils.cpp_extension.CUDAExtension`` rewrites sources through hipify on ROCm; this
project writes CDNA4 HIP directly, so the kernels are compiled by ``hipcc
--offload-arch=gfx950`` as-is and only linked against libtorch here.

    python -m llm_in_practise_amd.csrc.build          # both extensions, in-tree
    python -m llm_in_practise_amd.csrc.build --hip    # HIP kernels only

Objects are cached under ``build/native`` by (source mtime, flags); compiles run in
parallel (``MAX_JOBS``, default 8).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import importlib
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("LIPA_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX")


def _torch_flags():
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths(device_type="cuda") if "device_type" in ce.include_paths.__code__.co_varnames else ce.include_paths(True)
    libs = ce.library_paths(device_type="cuda") if "device_type" in ce.library_paths.__code__.co_varnames else ce.library_paths(True)
    import torch
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, libs, abi


def _run(cmd: list[str], cwd=None):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def _stamp(path: str, flags: list[str], deps: list[str]) -> str:
    h = hashlib.sha1(" ".join(flags).encode())
    for p in [path] + deps:
        h.update(p.encode())
        h.update(str(os.path.getmtime(p)).encode())
    return h.hexdigest()[:16]


def _compile(src: str, flags: list[str], compiler: list[str], deps: list[str]) -> str:
    os.makedirs(BUILD, exist_ok=True)
    base = os.path.relpath(src, PKG).replace(os.sep, "_")
    obj = os.path.join(BUILD, f"{base}.{_stamp(src, flags, deps)}.o")
    if not os.path.exists(obj):
        _run(compiler + flags + ["-c", src, "-o", obj + ".tmp"])
        os.replace(obj + ".tmp", obj)
    return obj


def build_hip_extension(jobs: int | None = None, verbose: bool = True) -> str:
    inc, libs, abi = _torch_flags()
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    kdir = os.path.join(HERE, "kernels")
    headers = sorted(glob.glob(os.path.join(kdir, "*.h")))
    kflags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
              "-ffp-contract=fast", f"-I{kdir}"]
    # LIPA_HIP_DEFINES="-DNAME ...": A/B builds of kernel variants (scripts/gpu_r6_ab_build.sh); never set by default
    kflags += [d for d in os.environ.get("LIPA_HIP_DEFINES", "").split() if d.startswith("-D")]
    bflags = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
              "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C",
              f"-I{sysconfig.get_paths()['include']}", f"-I{ROCM}/include"] + [f"-I{p}" for p in inc]
    srcs = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    jobs = jobs or int(os.environ.get("MAX_JOBS", "8"))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, kflags, [hipcc], headers) for s in srcs]
        futs.append(ex.submit(_compile, os.path.join(HERE, "bindings.cpp"), bflags, ["g++"], []))
        objs = [f.result() for f in futs]
    out = os.path.join(PKG, f"_C{EXT_SUFFIX}")
    link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out + ".tmp"] + objs
    link += [f"-L{p}" for p in libs] + [f"-Wl,-rpath,{p}" for p in libs]
    link += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip", "-lamdhip64", "-lhipblaslt"]
    _run(link)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"[lipa build] {os.path.relpath(out, ROOT)} ({len(srcs)} HIP sources, {ARCH})")
    return out


def build_cpu_extension(verbose: bool = True):
    """Build (if needed) and import ``llm_in_practise_amd._cpu``."""
    inc, libs, abi = _torch_flags()
    srcs = sorted(glob.glob(os.path.join(HERE, "cpu", "*.cpp")))
    flags = ["-O3", "-std=c++17", "-fPIC", "-fopenmp", "-march=native", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
             "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_cpu",
             f"-I{sysconfig.get_paths()['include']}"] + [f"-I{p}" for p in inc]
    hdrs = sorted(glob.glob(os.path.join(HERE, "cpu", "*.h")))
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags, ["g++"], hdrs), srcs))
    out = os.path.join(PKG, f"_cpu{EXT_SUFFIX}")
    link = ["g++", "-shared", "-fPIC", "-fopenmp", "-o", out + ".tmp"] + objs
    link += [f"-L{p}" for p in libs if "rocm" not in p] + [f"-Wl,-rpath,{p}" for p in libs if "rocm" not in p]
    link += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python"]
    _run(link)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"[lipa build] {os.path.relpath(out, ROOT)} ({len(srcs)} C++ sources)")
    importlib.invalidate_caches()
    return importlib.import_module("llm_in_practise_amd._cpu")


def build_sanitizer_harness(kind: str = "address") -> str:
    """Build ``tests/native/sanitize_host.cpp`` (the host runtime sources without bindings) as an
    executable under ``-fsanitize=address,undefined`` (``kind="address"``) or ``-fsanitize=thread``.
    Host code only: GPU sanitizers / XNACK are not available on the MI355X pool.  Returns the path;
    rebuilt only when a source is newer than the binary."""
    inc, libs, abi = _torch_flags()
    src = os.path.join(ROOT, "tests", "native", "sanitize_host.cpp")
    deps = [src] + sorted(glob.glob(os.path.join(HERE, "cpu", "*.cpp")))
    san = {"address": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
           "thread": ["-fsanitize=thread"]}[kind]
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(BUILD, f"sanitize_host_{kind}")
    if os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    lib_dirs = [p for p in libs if "rocm" not in p]
    # no OpenMP here: libgomp is not TSan-instrumented, so the OMP pragmas compile to serial loops
    cmd = ["g++", "-O1", "-g", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
           "-DTORCH_EXTENSION_NAME=_sanitize", f"-I{sysconfig.get_paths()['include']}", "-Wno-unknown-pragmas"]
    cmd += san + [f"-I{p}" for p in inc] + [src, "-o", out + ".tmp"]
    cmd += [f"-L{p}" for p in lib_dirs] + [f"-Wl,-rpath,{p}" for p in lib_dirs]
    cmd += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", f"-L{sysconfig.get_config_var('LIBDIR')}",
            f"-lpython{sysconfig.get_python_version()}", "-lpthread"]
    _run(cmd)
    os.replace(out + ".tmp", out)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--hip", action="store_true")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--sanitize", choices=["address", "thread"], help="build + run the host sanitizer harness")
    a = ap.parse_args(argv)
    if a.clean:
        shutil.rmtree(BUILD, ignore_errors=True)
    if a.sanitize:
        exe = build_sanitizer_harness(a.sanitize)
        return subprocess.call([exe])
    both = not (a.hip or a.cpu)
    if a.hip or both:
        build_hip_extension()
    if a.cpu or both:
        build_cpu_extension()


if __name__ == "__main__":
    sys.exit(main())
