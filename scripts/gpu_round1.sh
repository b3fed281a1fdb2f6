#!/bin/bash
# First GPU session: kernel numerics, smoke, stock vs native bench (each step time-limited;
# stop at the first crash/timeout, keep going only over ordinary test failures).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 300 python bench.py --impl torch --steps 10 --warmup 3 > $O/bench_torch1.log 2>&1
rc=$?; echo "bench_torch rc=$rc" | tee -a $O/status.txt; ok $rc || exit $rc
timeout -k 10 420 python -m pytest tests/test_kernels_gpu.py -q -m gpu > $O/pytest_gpu1.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a $O/status.txt; ok $rc || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > $O/smoke1.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a $O/status.txt; ok $rc || exit $rc
timeout -k 10 300 python bench.py --impl native --steps 10 --warmup 3 > $O/bench_native1.log 2>&1
rc=$?; echo "bench_native rc=$rc" | tee -a $O/status.txt
tail -n 3 $O/*.log
exit 0
