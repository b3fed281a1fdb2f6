#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_gpu4 timeout -k 10 420 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x; ok $? || exit 1
step convbench4 timeout -k 10 600 python scripts/bench_conv.py --json $O/convbench4.json; ok $? || exit 1
step bench_native4 timeout -k 10 300 python bench.py --impl native --steps 20 --warmup 5
exit 0
