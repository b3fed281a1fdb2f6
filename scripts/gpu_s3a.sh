#!/bin/bash
# Session-3 check of HEAD: GPU tests, smoke, bf16/fp8 bench, rocprof kernel stats.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_s3a timeout -k 10 500 python -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread; ok $? || exit 1
step smoke_s3a timeout -k 10 200 python __graft_entry__.py smoke || exit 1
step bench_s3a timeout -k 10 200 python bench.py --steps 20 --warmup 5 || exit 1
step bench_fp8_s3a timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp8 || exit 1
step bench152_s3a timeout -k 10 200 python bench.py --arch resnet152 --steps 10 --warmup 3 || exit 1
cd /tmp && export TMPDIR=/tmp
step prof_s3a timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s3a -o run -- python3 $R/bench.py --steps 5 --warmup 3
exit 0
