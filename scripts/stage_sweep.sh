#!/bin/bash
# Pipeline-depth sweep: conv tests + conv microbench with 2-stage vs 3-stage LDS pipelines.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
export PDT_NT_STAGES=3,3,3 PDT_TN_STAGES=3,3
step pytest_st3 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "conv or block or resnet" || exit 1
step convbench_st3 timeout -k 10 300 python scripts/bench_conv.py || exit 1
export PDT_NT_STAGES=2,3,2 PDT_TN_STAGES=3,2
step convbench_st232 timeout -k 10 300 python scripts/bench_conv.py || exit 1
unset PDT_NT_STAGES PDT_TN_STAGES
step convbench_st2 timeout -k 10 300 python scripts/bench_conv.py || exit 1
exit 0
