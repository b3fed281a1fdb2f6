#!/bin/bash
# ResNet-50 fp8 training parity sweep (diagnostics for tests/test_convergence_gpu.py): runs
# scripts/train_parity.py at the test's config for each variant given as an argument
# ("bf16", "all", "fwd", "fwd+dgrad"; a variant may repeat), one JSON per run under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-fp8sweep}
i=0
for v in "$@"; do
  i=$((i+1))
  case $v in
    bf16) args="" ;;
    *) args="--fp8 --fp8-parts $v" ;;
  esac
  timeout -k 10 240 python -u scripts/train_parity.py --arch resnet50 --image 112 --batch 64 --lr 0.004 \
      --steps 200 $args --json "gpurun_out/${TAG}_${i}.json" > "gpurun_out/${TAG}_${i}.log" 2>&1 || exit 1
  echo "run $i ($v) done"
done
