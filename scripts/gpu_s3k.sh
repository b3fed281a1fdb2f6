#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
cd /tmp && export TMPDIR=/tmp
step prof_s3k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s3k -o run -- python3 $R/bench.py --steps 5 --warmup 3
