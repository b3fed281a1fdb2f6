#!/bin/bash
# re-verification with device kernargs on by default: GPU tests (incl. graph capture), smoke, benches
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step g_pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
step g_smoke timeout -k 10 200 python __graft_entry__.py smoke || exit 1
step g_bench timeout -k 10 200 python bench.py --json-out $O/s5_g_bench.json || exit 1
step g_c_graph timeout -k 10 200 python bench.py --arch resnet18 --image-size 32 --num-classes 10 --graph --steps 100 --warmup 10 --json-out $O/s5_g_c_graph.json || exit 1
step g_c_eager timeout -k 10 200 python bench.py --arch resnet18 --image-size 32 --num-classes 10 --steps 100 --warmup 10 --json-out $O/s5_g_c_eager.json || exit 1
step g_r152 timeout -k 10 250 python bench.py --arch resnet152 --steps 15 --warmup 3 --json-out $O/s5_g_r152.json || exit 1
