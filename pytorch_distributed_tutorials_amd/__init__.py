"""pytorch_distributed_tutorials_amd -- an MI355X-native distributed data-parallel CNN trainer.

Same capabilities as chkda/pytorch-distributed-tutorials ``resnet/main.py``
(DDP ResNet training with a torchrun launcher, DistributedSampler, periodic
rank-0 evaluation and ``module.``-prefixed state_dict checkpoints), re-designed
for AMD Instinct MI355X (gfx950): NHWC bf16 fused HIP kernels, a C++ gradient
reducer over RCCL/xGMI and a flat fused SGD.

Layout:
  models/    ResNet family (torchvision naming)
  ops/       fused ops -> HIP kernels (csrc/kernels)
  parallel/  process groups, RCCL communicator, DDP wrapper + reducer
  optim/     flat-buffer fused SGD
  data/      DistributedSampler, synthetic device data, CIFAR-10
  utils/     env contract, seeding, checkpoints, profiling
"""
import os as _os

# Kernel arguments in device memory: the HIP runtime then skips the per-launch host-to-device
# kernarg copy.  Measured on MI355X (profiles/r1s5_runtime_knobs.jsonl): host-bound ResNet-18 /
# CIFAR step 87.3k -> 91.3k img/s, GPU-bound ResNet-50 step unchanged.  Read when the HIP
# runtime initialises (first device call), so it must be set before that; set it to 0 to opt out.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

__version__ = "0.1.0"
