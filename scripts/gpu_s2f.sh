#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_s2f timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py -v --timeout 120 --timeout-method thread; ok $? || exit 1
step diag_fp8_c timeout -k 10 200 python scripts/diag_fp8.py || exit 1
exit 0
