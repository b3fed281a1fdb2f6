#!/bin/bash
# final HEAD check of the session: GPU tests, smoke, headline bench, extra configs (R18 @224, R50 b512)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step e_pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
step e_smoke timeout -k 10 200 python __graft_entry__.py smoke || exit 1
step e_bench timeout -k 10 200 python bench.py --json-out $O/s5_e_bench.json || exit 1
step e_r18 timeout -k 10 200 python bench.py --arch resnet18 --steps 30 --warmup 5 --json-out $O/s5_e_r18.json || exit 1
step e_b512 timeout -k 10 250 python bench.py --batch 512 --steps 20 --warmup 3 --json-out $O/s5_e_b512.json || exit 1
