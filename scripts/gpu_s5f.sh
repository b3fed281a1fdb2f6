#!/bin/bash
# runtime knob A/B: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs default
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step f_base timeout -k 10 200 python bench.py --steps 40 --warmup 5 --json-out $O/s5_f_base.json || exit 1
step f_dka timeout -k 10 200 env HIP_FORCE_DEV_KERNARG=1 python bench.py --steps 40 --warmup 5 --json-out $O/s5_f_dka.json || exit 1
step f_base2 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --json-out $O/s5_f_base2.json || exit 1
step f_dka2 timeout -k 10 200 env HIP_FORCE_DEV_KERNARG=1 python bench.py --steps 40 --warmup 5 --json-out $O/s5_f_dka2.json || exit 1
step f_c_base timeout -k 10 200 python bench.py --arch resnet18 --image-size 32 --num-classes 10 --steps 100 --warmup 10 --json-out $O/s5_f_c_base.json || exit 1
step f_c_dka timeout -k 10 200 env HIP_FORCE_DEV_KERNARG=1 python bench.py --arch resnet18 --image-size 32 --num-classes 10 --steps 100 --warmup 10 --json-out $O/s5_f_c_dka.json || exit 1
