#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for sh in 256x56x56x64x1x1x1x0 512x28x28x128x1x1x1x0; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bn_$sh -o run -- python3 $R/scripts/bench_conv.py --only $sh --bn --iters 5 > $O/prof_bn_$sh.log 2>&1 || exit 1
done
exit 0
