#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
BENCH_ARGS="--bn" SHAPES="64x56x56x256x1x1x1x0 256x56x56x64x1x1x1x0" bash scripts/pmc_conv.sh pmc_s2o || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc_s2o > gpurun_out/pmc_s2o_summary.txt 2>&1
exit 0
