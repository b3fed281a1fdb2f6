#!/bin/bash
# round-end rehearsal on HEAD: full GPU test suite, smoke(), headline bench
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step a_pytest timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
step a_smoke timeout -k 10 200 python __graft_entry__.py smoke || exit 1
step a_bench timeout -k 10 200 python bench.py || exit 1
step a_bench40 timeout -k 10 200 python bench.py --steps 40 --warmup 5
