#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
SHAPES="256x14x14x256x3x3x1x1 64x56x56x64x3x3x1x1 64x56x56x256x1x1x1x0" bash scripts/pmc_conv.sh pmc_s3h
echo "pmc rc=$?" >> $O/status.txt
python scripts/pmc_summary.py $O/pmc_s3h > $O/pmc_s3h_summary.txt 2>&1
