#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step diag_cpu_s3g timeout -k 10 200 python scripts/diag_cpu.py || exit 1
