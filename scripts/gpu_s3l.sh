#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_s3l timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -k "stem or conv_fwd or resnet" || exit 1
step convbench_s3l timeout -k 10 300 python scripts/bench_conv.py --only 3x224x224x64x7x7x2x3 || exit 1
step bench_s3l timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
