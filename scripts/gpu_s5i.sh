#!/bin/bash
# BN forward apply with two grid-stride iterations in flight: kernel tests, bench, kernel stats
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step i_pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
step i_bench timeout -k 10 200 python bench.py --steps 40 --warmup 5 --json-out $O/s5_i_bench.json || exit 1
step i_bench2 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --json-out $O/s5_i_bench2.json || exit 1
cd /tmp && export TMPDIR=/tmp
step i_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s5i -o run -- python3 $R/bench.py --steps 5 --warmup 3
