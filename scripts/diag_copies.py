#!/usr/bin/env python3
"""Where do the small device-to-device copies / fills / adds of a ResNet-50 step come from?

Profiles one warm native training step with torch.profiler (CPU ops + device activity,
Python stacks) and prints, for every aten op that moves bytes without computing
(copy_, fill_, zero_, add_ of grads, clone, to), its count per step and the Python
frames that issued it.
"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd import ops  # noqa: E402
from pytorch_distributed_tutorials_amd.models import build_model  # noqa: E402
from pytorch_distributed_tutorials_amd.optim import SGD  # noqa: E402
from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    batch = int(os.environ.get("BATCH", "64"))
    model = build_model("resnet50", num_classes=1000, impl="native").to(dev)
    model.set_impl("native")
    ddp = DistributedDataParallel(model)
    opt = SGD(ddp.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-5)
    crit = ops.CrossEntropyLoss()
    x = torch.randn(batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (batch,), device=dev)

    def step():
        opt.zero_grad()
        loss = crit(ddp(x), y)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    watch = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::clone", "aten::to", "aten::_to_copy",
             "aten::add_", "aten::add", "aten::mul", "aten::div_", "aten::sum", "aten::zeros")
    by = collections.Counter()
    for ev in prof.events():
        if ev.name in watch:
            frames = [f for f in (ev.stack or []) if "pytorch_distributed_tutorials_amd" in f or "diag_" in f]
            by[(ev.name, " <- ".join(frames[:3]))] += 1
    for (name, st), n in by.most_common(40):
        print(f"{n:4d}  {name:16s} {st}")
    print()
    print(prof.key_averages().table(sort_by="device_time_total", row_limit=30))


if __name__ == "__main__":
    main()
