#!/bin/bash
# N>1 bench path rehearsal on a one-GPU box (2 ranks share cuda:0 over gloo, native kernels + reducer),
# plus the eager vs graph ResNet-50 comparison at HEAD
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step b_n2 timeout -k 10 300 env MASTER_PORT=29533 python bench.py --gpus 2 --backend gloo --share-device --steps 10 --warmup 3 --json-out $O/s5_b_n2_shared_gloo.json || exit 1
step b_graph timeout -k 10 200 python bench.py --graph --steps 40 --warmup 5 --json-out $O/s5_b_graph.json || exit 1
step b_eager timeout -k 10 200 python bench.py --steps 40 --warmup 5 --json-out $O/s5_b_eager.json || exit 1
