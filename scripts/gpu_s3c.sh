#!/bin/bash
# wgrad staged epilogue A/B (PDT_TN_STAGED), split caps, BN reduce stage1/2: tests, conv bench, bench.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_s3c timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -k "bn or wgrad or sink or resnet18 or residual or captured" || exit 1
step bench_s3c timeout -k 10 200 python bench.py --steps 20 --warmup 5 || exit 1
PDT_TN_STAGED=0 step bench_s3c_unstaged timeout -k 10 200 python bench.py --steps 20 --warmup 5 || exit 1
step convbench_s3c timeout -k 10 300 python scripts/bench_conv.py || exit 1
PDT_TN_STAGED=0 step convbench_s3c_unstaged timeout -k 10 300 python scripts/bench_conv.py || exit 1
step convbench_s3c_det timeout -k 10 300 python scripts/bench_conv.py --det || exit 1
PDT_WGRAD_CAP_MB=64,64 step convbench_s3c_cap64 timeout -k 10 300 python scripts/bench_conv.py || exit 1
exit 0
