#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_s2p timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread; ok $? || exit 1
step convbench_s2p timeout -k 10 300 python scripts/bench_conv.py --bn || exit 1
step bench_s2p timeout -k 10 200 python bench.py --steps 20 --warmup 5 || exit 1
step bench_fp8_s2p timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp8 || exit 1
exit 0
