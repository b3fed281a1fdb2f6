#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_gpu3 timeout -k 10 420 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x; ok $? || exit 1
step bench_native3 timeout -k 10 300 python bench.py --impl native --steps 20 --warmup 5; ok $? || exit 1
step convbench3 timeout -k 10 600 python scripts/bench_conv.py --torch --json $O/convbench3.json; ok $? || exit 1
step bench_torch_bm3 timeout -k 10 400 python bench.py --impl torch --steps 20 --warmup 5 --cudnn-benchmark; ok $? || exit 1
cd /tmp && export TMPDIR=/tmp
step prof_native3 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_native3 -o run -- python3 $R/bench.py --impl native --steps 3 --warmup 2
exit 0
