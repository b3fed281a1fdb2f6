#!/bin/bash
# in-step sweep of the wgrad split-K atomic-traffic cap
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
for cap in 32 8 16 24 48; do
  PDT_WGRAD_CAP_MB=$cap,64 step bench_s3d_cap$cap timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
done
exit 0
