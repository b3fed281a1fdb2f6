#!/bin/bash
# Generic GPU check: kernel tests, conv microbench, native bench (+ optional rocprof).
# usage: bash scripts/gpu_check.sh TAG [prof]
TAG=${1:-x}
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_$TAG timeout -k 10 420 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x; ok $? || exit 1
step bench_$TAG timeout -k 10 300 python bench.py --impl native --steps 20 --warmup 5; ok $? || exit 1
step convbench_$TAG timeout -k 10 600 python scripts/bench_conv.py; ok $? || exit 1
if [ "$2" = "prof" ]; then
  cd /tmp && export TMPDIR=/tmp
  step prof_$TAG timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 $R/bench.py --impl native --steps 3 --warmup 2
fi
exit 0
