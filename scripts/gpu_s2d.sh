#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step convbench_s2d timeout -k 10 300 python scripts/bench_conv.py --fp8 || exit 1
cd /tmp && export TMPDIR=/tmp
step prof_fp8_s2d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp8_s2d -o run -- python3 $R/bench.py --steps 3 --warmup 2 --fp8
exit 0
