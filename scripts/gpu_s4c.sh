#!/bin/bash
# per-row-tile BN partials + fence-free last-block reductions: numerics, bench, conv microbench, copy sources
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step c_pytest timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step c_bench timeout -k 10 200 python bench.py --steps 40 --warmup 5 || exit 1
step c_bench_fp8 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --fp8 || exit 1
step c_convbench timeout -k 10 400 python scripts/bench_conv.py --bn || exit 1
step c_copies timeout -k 10 300 python scripts/diag_copies.py
