#!/bin/bash
# end-of-session check of the in-tree extension the driver will load: GPU tests + smoke + bench
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step j_pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step j_smoke timeout -k 10 200 python __graft_entry__.py smoke || exit 1
step j_bench timeout -k 10 200 python bench.py --json-out $O/s5_j_bench.json || exit 1
