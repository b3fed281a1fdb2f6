#!/bin/bash
# GPU session 2: numerics (minus the RCCL test), smoke, native bench, rocprof kernel stats, RCCL test last.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_gpu2 timeout -k 10 420 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "not rccl"; ok $? || exit 1
step smoke2 timeout -k 10 200 python __graft_entry__.py smoke; ok $? || exit 1
step bench_native2 timeout -k 10 300 python bench.py --impl native --steps 10 --warmup 3; ok $? || exit 1
cd /tmp && export TMPDIR=/tmp
step prof_native2 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_native2 -o run -- python3 $R/bench.py --impl native --steps 3 --warmup 2; ok $? || exit 1
step prof_torch2 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_torch2 -o run -- python3 $R/bench.py --impl torch --steps 3 --warmup 2; ok $? || exit 1
cd "$R"
step pytest_rccl2 timeout -k 10 120 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "rccl"
tail -n 2 $O/*2.log
exit 0
