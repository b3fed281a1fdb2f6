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
__version__ = "0.1.0"
