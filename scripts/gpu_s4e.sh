#!/bin/bash
# elementwise BN passes: fixed channel group per thread + two vectors per trip
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step e_pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step e_bench timeout -k 10 200 python bench.py --steps 40 --warmup 5 || exit 1
step e_bench2 timeout -k 10 200 python bench.py --steps 40 --warmup 5 || exit 1
cd /tmp && export TMPDIR=/tmp
step e_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s4e -o run -- python3 $R/bench.py --steps 5 --warmup 3
