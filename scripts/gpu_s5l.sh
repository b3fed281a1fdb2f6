#!/bin/bash
# per-pass BN grid caps (residual forward apply 32768): GPU tests, bench x2, kernel stats
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step l_pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step l_smoke timeout -k 10 200 python __graft_entry__.py smoke || exit 1
step l_bench timeout -k 10 200 python bench.py --steps 40 --warmup 5 --json-out $O/s5_l_bench.json || exit 1
step l_bench2 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --json-out $O/s5_l_bench2.json || exit 1
cd /tmp && export TMPDIR=/tmp
step l_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s5l -o run -- python3 $R/bench.py --steps 10 --warmup 3
