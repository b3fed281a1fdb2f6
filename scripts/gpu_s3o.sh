#!/bin/bash
# per-shape NT tile policy study: default vs wide tile disabled vs wide tile forced
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step o_def timeout -k 10 300 python scripts/bench_conv.py --bn || exit 1
PDT_NT_TILE=1 step o_t1 timeout -k 10 300 python scripts/bench_conv.py --bn || exit 1
PDT_NT_TILE=2 step o_t2 timeout -k 10 300 python scripts/bench_conv.py --bn || exit 1
PDT_NT_STAGES=3,3,3 step o_s3 timeout -k 10 300 python scripts/bench_conv.py --bn || exit 1
