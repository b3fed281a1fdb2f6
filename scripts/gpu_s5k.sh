#!/bin/bash
# grid-cap A/B of the streaming BN passes (PDT_EW_BLOCKS): per-kernel stats for each cap
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
for cap in 4096 8192 16384 32768; do
  export PDT_EW_BLOCKS=$cap
  step k_prof_$cap timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s5k_$cap -o run -- python3 $R/bench.py --steps 10 --warmup 3 || exit 1
done
