#!/bin/bash
# fp8 MFMA probe, 2-rank DDP on one GPU, ResNet-152 / ResNet-18@32 benches.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_s2b timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_ddp_gpu.py -v --timeout 120 --timeout-method thread; ok $? || exit 1
step bench_r152_s2b timeout -k 10 300 python bench.py --arch resnet152 --steps 10 --warmup 3 || exit 1
step bench_r18c_s2b timeout -k 10 300 python bench.py --arch resnet18 --image-size 32 --num-classes 10 --steps 50 --warmup 5 || exit 1
step bench_r152_torch_s2b timeout -k 10 400 python bench.py --arch resnet152 --impl torch --cudnn-benchmark --steps 10 --warmup 3 || exit 1
exit 0
