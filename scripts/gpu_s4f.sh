#!/bin/bash
# BN fwd hoist + trainer --graph: tests, bench, reference workload (ResNet-18 CIFAR trainer) eager vs graph
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step f_trgraph timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k trainer_graph -x -q --timeout 240 --timeout-method thread || exit 1
step f_pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit 1
step f_bench timeout -k 10 200 python bench.py --steps 40 --warmup 5 || exit 1
step f_bench2 timeout -k 10 200 python bench.py --steps 40 --warmup 5 || exit 1
T="-m pytorch_distributed_tutorials_amd.train --arch resnet18 --data synthetic-cifar --synthetic-samples 50000 --num-classes 10 --num_epochs 2 --eval-every 1 --log-every 49 --model_dir /tmp/pdt_ck"
step f_train_eager timeout -k 10 300 python $T || exit 1
step f_train_graph timeout -k 10 300 python $T --graph || exit 1
