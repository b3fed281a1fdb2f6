#!/bin/bash
# measurement batch for the docs: headline + configs, kernel stats profile
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step q_r50 timeout -k 10 200 python bench.py --steps 40 --warmup 5 || exit 1
step q_r50_fp8 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --fp8 || exit 1
step q_r50_fp8_b512 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --fp8 --batch 512 || exit 1
step q_r152 timeout -k 10 250 python bench.py --arch resnet152 --steps 15 --warmup 3 || exit 1
step q_r18c timeout -k 10 200 python bench.py --arch resnet18 --image-size 32 --num-classes 10 --steps 50 --warmup 5 || exit 1
step q_r50_wire_bf16 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --wire-dtype bf16 || exit 1
step q_cpu timeout -k 10 200 python scripts/diag_cpu.py || exit 1
cd /tmp && export TMPDIR=/tmp
step q_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s3q -o run -- python3 $R/bench.py --steps 5 --warmup 3
