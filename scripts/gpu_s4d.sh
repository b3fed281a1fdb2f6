#!/bin/bash
# wgrad side-stream hand-offs batched per block: A/B bench, GPU tests touching streams, kernel stats
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step d_pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step d_bench_b1 timeout -k 10 200 python bench.py --steps 40 --warmup 5 || exit 1
step d_bench_b0 timeout -k 10 200 env PDT_WGRAD_BATCH=0 python bench.py --steps 40 --warmup 5 || exit 1
step d_bench_b1r timeout -k 10 200 python bench.py --steps 40 --warmup 5 || exit 1
step d_r152 timeout -k 10 250 python bench.py --arch resnet152 --steps 15 --warmup 3 || exit 1
cd /tmp && export TMPDIR=/tmp
step d_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s4d -o run -- python3 $R/bench.py --steps 5 --warmup 3
