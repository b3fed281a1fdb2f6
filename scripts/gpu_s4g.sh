#!/bin/bash
# epilogue batch depth A/B (4 / 8 / 16 chunks in flight): conv microbench with BN-fused dgrad + bench
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step g_cb4 timeout -k 10 300 python scripts/bench_conv.py --bn || exit 1
step g_cb8 timeout -k 10 300 python build/it8/scripts/bench_conv.py --bn || exit 1
step g_cb16 timeout -k 10 300 python build/it16/scripts/bench_conv.py --bn || exit 1
step g_b4 timeout -k 10 200 python bench.py --steps 40 --warmup 5 || exit 1
step g_b8 timeout -k 10 200 python build/it8/bench.py --steps 40 --warmup 5 || exit 1
step g_b16 timeout -k 10 200 python build/it16/bench.py --steps 40 --warmup 5 || exit 1
