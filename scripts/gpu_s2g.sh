#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
SHAPES="256x14x14x256x3x3x1x1 64x56x56x64x3x3x1x1 256x56x56x64x1x1x1x0" bash scripts/pmc_conv.sh pmc_s2g || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc_s2g > gpurun_out/pmc_s2g_summary.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python $R/bench.py --arch resnet152 --impl torch --steps 5 --warmup 2 > $R/gpurun_out/bench_r152_torch_s2g.log 2>&1
echo "r152 torch rc=$?" >> $R/gpurun_out/status.txt
exit 0
