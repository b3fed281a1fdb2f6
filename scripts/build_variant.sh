#!/bin/bash
# Build a tuning variant of the extension into build/<name>/ (a copy of the package + scripts with
# conv_igemm.hip recompiled with extra defines), for A/B runs:  python build/<name>/scripts/bench_conv.py
# usage: scripts/build_variant.sh NAME "-DMACRO=VALUE ..." ["kernel sources", default conv_igemm.hip]
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; DEFS=$2; SRC=${3:-conv_igemm.hip}
V=$R/build/$NAME; rm -rf $V; mkdir -p $V/obj
cp -r $R/pytorch_distributed_tutorials_amd $V/; cp -r $R/scripts $V/; cp $R/bench.py $R/build_native.py $V/
python3 - "$R" "$V" "$DEFS" "$SRC" <<'PY'
import os, sys, glob, subprocess, shlex
R, V, defs, srcname = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
sys.path.insert(0, R)
import build_native as b
import torch
abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
objs = sorted(glob.glob(os.path.join(R, "build", "native", "*.o")))
for srcname in srcname.split():
    src = os.path.join(R, "csrc", "kernels", srcname)
    obj = os.path.join(V, "obj", os.path.splitext(srcname)[0] + ".o")
    cmd = [b.HIPCC, "-std=c++17", "-fPIC", f"--offload-arch={b.ARCH}", "-D__HIP_PLATFORM_AMD__=1", "-O3",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", os.path.join(R, "csrc")] + shlex.split(defs) + ["-c", src, "-o", obj]
    subprocess.run(cmd, check=True)
    objs = [obj if o.endswith("kernels_" + srcname + ".o") else o for o in objs]
tdir = os.path.dirname(torch.__file__); tlib = os.path.join(tdir, "lib")
so = os.path.join(V, "pytorch_distributed_tutorials_amd", os.path.basename(b.out_path()))
link = [b.HIPCC, "-shared", "-fPIC", f"--offload-arch={b.ARCH}", "-o", so] + objs + [
    "-L", tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
    os.path.join(tlib, "librccl.so"), f"-Wl,-rpath,{tlib}", "-Wl,-rpath,/opt/rocm/lib"]
subprocess.run(link, check=True)
print("built", so)
PY
