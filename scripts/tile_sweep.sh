#!/bin/bash
# NT tile sweep: conv tests + conv microbench for each PDT_NT_TILE mode.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
for m in ${MODES:-1 2 3}; do
  export PDT_NT_TILE=$m
  step pytest_tile$m timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "conv or block or resnet" || exit 1
  step convbench_tile$m timeout -k 10 300 python scripts/bench_conv.py || exit 1
done
unset PDT_NT_TILE
step convbench_tile0 timeout -k 10 300 python scripts/bench_conv.py || exit 1
exit 0
