#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step r_cpu18 timeout -k 10 200 python scripts/diag_cpu.py resnet18 32 10 || exit 1
step r_r18g timeout -k 10 200 python bench.py --arch resnet18 --image-size 32 --num-classes 10 --steps 50 --warmup 5 --graph || exit 1
PDT_STEM_POOL=0 step r_r18np timeout -k 10 200 python bench.py --arch resnet18 --image-size 32 --num-classes 10 --steps 50 --warmup 5 || exit 1
cd /tmp && export TMPDIR=/tmp
step r_prof18 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r18 -o run -- python3 $R/bench.py --arch resnet18 --image-size 32 --num-classes 10 --steps 5 --warmup 3
