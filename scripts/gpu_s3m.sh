#!/bin/bash
# re-tune pipeline depth / tile knobs after the loader changes (in-step bench per setting)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step m_base timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
PDT_NT_STAGES=3,2,2 step m_st322 timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
PDT_NT_STAGES=2,3,2 step m_st232 timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
PDT_NT_STAGES=2,2,3 step m_st223 timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
PDT_NT_TILE=1 step m_tile1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
PDT_NT_TILE=2 step m_tile2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
PDT_TN_STAGES=3,3 step m_tn33 timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
PDT_TN_WIDE=1 step m_tnwide timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
step m_base2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
