#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
SHAPES="64x56x56x64x3x3x1x1 256x56x56x512x1x1x2x0 3x224x224x64x7x7x2x3" bash scripts/pmc_conv.sh pmc_s3n
echo "pmc rc=$?" >> $O/status.txt
python scripts/pmc_summary.py $O/pmc_s3n > $O/pmc_s3n_summary.txt 2>&1
timeout -k 10 300 python scripts/bench_conv.py --bn > $O/convbench_s3n_bn.log 2>&1
echo "convbench rc=$?" >> $O/status.txt
