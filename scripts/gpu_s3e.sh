#!/bin/bash
# fused stem BN/ReLU/max pool: full GPU suite, smoke, bench (fused vs PDT_STEM_POOL=0), graph bench, profile
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" | tee -a $O/status.txt; return $rc; }
step pytest_s3e timeout -k 10 500 python -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread || exit 1
step smoke_s3e timeout -k 10 200 python __graft_entry__.py smoke || exit 1
step bench_s3e timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
PDT_STEM_POOL=0 step bench_s3e_nopool timeout -k 10 200 python bench.py --steps 30 --warmup 5 || exit 1
step bench_s3e_graph timeout -k 10 200 python bench.py --steps 30 --warmup 5 --graph || exit 1
cd /tmp && export TMPDIR=/tmp
step prof_s3e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s3e -o run -- python3 $R/bench.py --steps 5 --warmup 3
