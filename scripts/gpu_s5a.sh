#!/bin/bash
# HEAD re-verification after container re-creation: GPU tests, smoke, bench configs, kernel stats
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step a_pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
step a_smoke timeout -k 10 200 python __graft_entry__.py smoke || exit 1
step a_bench timeout -k 10 200 python bench.py --steps 40 --warmup 5 --json-out $O/s5_a_bench.json || exit 1
step a_fp8 timeout -k 10 200 python bench.py --fp8 --steps 40 --warmup 5 --json-out $O/s5_a_fp8.json || exit 1
step a_r152 timeout -k 10 250 python bench.py --arch resnet152 --steps 15 --warmup 3 --json-out $O/s5_a_r152.json || exit 1
cd /tmp && export TMPDIR=/tmp
step a_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s5a -o run -- python3 $R/bench.py --steps 5 --warmup 3
