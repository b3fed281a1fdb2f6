#!/usr/bin/env python3
"""Build the native extension in-tree for gfx950 (MI355X).

    python build_native.py [--force] [--jobs N] [--debug] [--sanitize]

* every ``csrc/kernels/*.hip`` is compiled by ``hipcc --offload-arch=gfx950``
  WITHOUT PyTorch headers (fast, seconds per file);
* ``csrc/bindings.cpp``, ``csrc/comm/*.cpp`` and ``csrc/ddp/*.cpp`` are host C++
  compiled by hipcc against the installed PyTorch headers;
* everything is linked into ``pytorch_distributed_tutorials_amd/_C<EXT_SUFFIX>``
  against libtorch and the RCCL shipped inside the torch wheel, rpath'd to it.

Incremental: an object is rebuilt when its source or any header under csrc/ is
newer.  Works without a GPU (hipcc cross-compiles), so it runs in CI/CPU boxes.

``--sanitize``: a host-side AddressSanitizer + UndefinedBehaviorSanitizer build (``-O1 -g``,
``-fsanitize=address,undefined`` on the host compilation only -- GPU code stays uninstrumented)
into ``build/asan/_C*.so``, for the CPU tests of the host runtime (C++ reducer, bucket plan,
bindings' argument checks).  Run them with ``scripts/asan_cpu_tests.sh``: it preloads the clang
ASan runtime into python and points the loader at this build (``PDT_NATIVE_SO``).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shlex
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "pytorch_distributed_tutorials_amd")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, int(torch._C._GLIBCXX_USE_CXX11_ABI)


def out_path() -> str:
    return os.path.join(PKG, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _newest_header() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(shlex.quote(c) for c in cmd)}\n{r.stdout}")
    return r.stdout


SAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]


def asan_out_path() -> str:
    return os.path.join(ROOT, "build", "asan", "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def build(force: bool = False, jobs: int = 0, debug: bool = False, verbose: bool = True,
          sanitize: bool = False) -> str:
    tdir, tinc, abi = _torch_paths()
    bdir = os.path.join(ROOT, "build", "native_asan") if sanitize else BUILD
    os.makedirs(bdir, exist_ok=True)
    opt = ["-O0", "-g"] if debug else (["-O1", "-g"] + SAN_FLAGS if sanitize else ["-O3"])
    common = ["-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1",
              "-Wno-unused-result", "-Wno-unused-value"] + opt
    kern_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    host_srcs = [os.path.join(CSRC, "bindings.cpp")] + sorted(
        glob.glob(os.path.join(CSRC, "comm", "*.cpp")) + glob.glob(os.path.join(CSRC, "ddp", "*.cpp")))
    py_inc = sysconfig.get_paths()["include"]
    host_flags = common + [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
                           "-DTORCH_API_INCLUDE_EXTENSION_H", "-I", py_inc, "-I", CSRC,
                           "-I", "/opt/rocm/include"] + sum((["-I", i] for i in tinc), [])
    hdr_t = _newest_header()
    jobs_list = []
    objs = []
    for src in kern_srcs + host_srcs:
        rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
        obj = os.path.join(bdir, rel + ".o")
        objs.append(obj)
        stale = force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t)
        if not stale:
            continue
        if src.endswith(".hip"):
            cmd = [HIPCC] + common + [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", CSRC, "-c", src, "-o", obj]
        else:
            cmd = [HIPCC] + host_flags + ["-c", src, "-o", obj]
        jobs_list.append((src, cmd))
    n = jobs or min(8, os.cpu_count() or 4)
    if jobs_list:
        if verbose:
            print(f"[build_native] compiling {len(jobs_list)} file(s) for {ARCH} with {n} jobs", flush=True)
        with cf.ThreadPoolExecutor(n) as ex:
            futs = {ex.submit(_run, cmd): src for src, cmd in jobs_list}
            for f in cf.as_completed(futs):
                f.result()
                if verbose:
                    print(f"[build_native]   ok {os.path.relpath(futs[f], ROOT)}", flush=True)
    so = asan_out_path() if sanitize else out_path()
    os.makedirs(os.path.dirname(so), exist_ok=True)
    if force or jobs_list or not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(o) for o in objs):
        tlib = os.path.join(tdir, "lib")
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", so] + objs + [
            "-L", tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            os.path.join(tlib, "librccl.so"), f"-Wl,-rpath,{tlib}", "-Wl,-rpath,/opt/rocm/lib"]
        if sanitize:
            link += ["-fsanitize=address,undefined", "-shared-libsan"]
        _run(link)
        if verbose:
            print(f"[build_native] linked {os.path.relpath(so, ROOT)}", flush=True)
    return so


def ensure_built(verbose: bool = False) -> str:
    return build(force=False, verbose=verbose)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--sanitize", action="store_true", help="host ASan+UBSan build into build/asan/")
    a = ap.parse_args(argv)
    so = build(force=a.force, jobs=a.jobs, debug=a.debug, sanitize=a.sanitize)
    print(so)
    return 0


if __name__ == "__main__":
    sys.exit(main())
