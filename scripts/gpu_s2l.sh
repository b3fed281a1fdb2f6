#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_s2l timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "augment"; ok $? || exit 1
step train_fp8_s2l timeout -k 10 300 python -m pytorch_distributed_tutorials_amd.train --arch resnet18 --data synthetic-cifar --num-classes 10 --synthetic-samples 4096 --num_epochs 2 --eval-every 1 --dtype fp8 --log-every 8 --model_dir /tmp/pdt_ckpt || exit 1
exit 0
