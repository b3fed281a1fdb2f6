set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for p in fwd fwd+dgrad all; do
  timeout -k 10 300 python -u scripts/train_parity.py --arch resnet50 --image 112 --batch 64 --lr 0.004 --steps 200 --repeats 3 --fp8 --fp8-parts $p --json gpurun_out/r8a_$p.json > gpurun_out/r8a_$p.log 2>&1 || exit 1
done
