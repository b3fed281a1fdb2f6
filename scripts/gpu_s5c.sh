#!/bin/bash
# HBM bytes per kernel over a ResNet-50 bf16 step: FETCH_SIZE and WRITE_SIZE in separate passes
# (FETCH_SIZE takes 3 TCC counters, WRITE_SIZE 2: one pass cannot hold both)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step c_fetch timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_s5c_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 || exit 1
step c_write timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_s5c_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 || exit 1
