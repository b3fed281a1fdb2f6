#!/usr/bin/env python3
"""fp8 forward determinism: the same ResNet-50 fp8 forward (no optimizer step) repeated; every
loss after the delayed-scaling warm-up must be bit-identical.  Prints the losses per setting."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytorch_distributed_tutorials_amd.ops.fused as fused  # noqa: E402
from pytorch_distributed_tutorials_amd import ops  # noqa: E402
from pytorch_distributed_tutorials_amd.models import build_model  # noqa: E402
from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel  # noqa: E402


def main():
    gpu = torch.device("cuda:0")
    torch.manual_seed(0)
    m = build_model("resnet50", num_classes=10, impl="native").to(gpu).set_impl("native")
    ddp = DistributedDataParallel(m)
    x = torch.randn(16, 3, 64, 64, device=gpu)
    yl = torch.randint(0, 10, (16,), device=gpu)
    ops.set_fp8(True)
    for bwd8 in (False, True, False, True):
        fused._FP8_BWD = bwd8
        ls = []
        for _ in range(4):
            ddp.space.zero_grad()
            loss = ops.cross_entropy(ddp(x), yl)
            loss.backward()
            ls.append(loss.item())
        print(f"kmin={fused._FP8_KMIN} fp8_bwd={bwd8} losses={ls}", flush=True)
    fused._FP8_BWD = True
    ls = []
    with torch.no_grad():
        for _ in range(4):
            ls.append(ops.cross_entropy(ddp(x), yl).item())
    print(f"no-grad forward losses={ls}", flush=True)


if __name__ == "__main__":
    main()
