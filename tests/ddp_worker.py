"""Multi-process DDP worker used by tests/test_ddp_cpu.py (gloo, CPU).

Launched by ``pytorch_distributed_tutorials_amd.launch --nproc_per_node=N``.
Trains the same model with (a) our DistributedDataParallel + fused SGD and
(b) torch.nn.parallel.DistributedDataParallel + torch.optim.SGD from identical
initial weights on rank-dependent synthetic batches, interleaving a rank-0-only
evaluation pass (the reference's eval pattern, resnet/main.py:109-112), then
dumps checksums / max differences as JSON for the test to assert on.
"""
import argparse
import copy
import json
import os
import sys

import torch
import torch.distributed as dist
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_tutorials_amd import ops  # noqa: E402
from pytorch_distributed_tutorials_amd.models import build_model  # noqa: E402
from pytorch_distributed_tutorials_amd.optim import SGD  # noqa: E402
from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel, init_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--impl", default="torch")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--pyreducer", action="store_true")
    a = ap.parse_args()
    torch.set_num_threads(2)
    env = init_distributed("gloo")
    rank, world = env.rank, env.world_size
    if a.pyreducer:
        import pytorch_distributed_tutorials_amd.parallel.ddp as ddpmod
        ddpmod.native_available = lambda: False

    torch.manual_seed(1234 + rank)  # deliberately different init per rank: DDP must broadcast rank 0's
    base = build_model(a.arch, num_classes=10)
    ref_model = copy.deepcopy(base)
    ours = DistributedDataParallel(copy.deepcopy(base).set_impl(a.impl), bucket_cap_mb=1.0)
    # separate process group: the two wrappers' collective streams must not interleave
    # (rank 0's extra eval forwards shift each wrapper's sequence independently)
    theirs = nn.parallel.DistributedDataParallel(ref_model, bucket_cap_mb=1.0,
                                                 process_group=dist.new_group(backend="gloo"))
    opt_o = SGD(ours.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    opt_t = torch.optim.SGD(theirs.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    crit_o = ops.CrossEntropyLoss() if a.impl == "native" else nn.CrossEntropyLoss()
    crit_t = nn.CrossEntropyLoss()

    # run the two wrappers one after the other (same data stream) so their collective
    # sequences never wait on each other across process groups
    evaluated = 0
    for model, opt, crit in ((ours, opt_o, crit_o), (theirs, opt_t, crit_t)):
        g = torch.Generator().manual_seed(99 + rank)
        for step in range(a.steps):
            # rank-0-only eval at the reference's points: before the first training step
            # (epoch 0) and later, after torch DDP's iteration-1 bucket rebuild.  (An eval
            # right after iteration 0 mis-pairs torch DDP's own rebuild broadcast.)
            if rank == 0 and step in (0, 2):
                model.eval()
                with torch.no_grad():
                    model(torch.randn(2, 3, 32, 32))
                evaluated += 1
            x = torch.randn(4, 3, 32, 32, generator=g)
            y = torch.randint(0, 10, (4,), generator=g)
            model.train()
            opt.zero_grad()
            loss = crit(model(x), y)
            loss.backward()
            opt.step()

    res = {"rank": rank, "world": world, "evaluated": evaluated,
           "bucket_info": ours.bucket_info(),
           "ours_checksum": float(sum(p.detach().double().sum() for p in ours.parameters())),
           "theirs_checksum": float(sum(p.detach().double().sum() for p in theirs.parameters()))}
    diffs = []
    for (n1, p1), (n2, p2) in zip(ours.module.named_parameters(), theirs.module.named_parameters()):
        assert n1 == n2
        diffs.append((p1.detach() - p2.detach()).abs().max().item())
    res["max_param_diff_vs_torch_ddp"] = max(diffs)
    bdiffs = []
    for (n1, b1), (n2, b2) in zip(ours.module.named_buffers(), theirs.module.named_buffers()):
        bdiffs.append((b1.double() - b2.double()).abs().max().item())
    res["max_buffer_diff_vs_torch_ddp"] = max(bdiffs)
    res["keys_equal"] = list(ours.state_dict().keys()) == list(theirs.state_dict().keys())
    if hasattr(ours.reducer, "last_launch_order"):
        res["launch_order"] = list(ours.reducer.last_launch_order())
    # cross-rank equality of our parameters
    t = torch.tensor([res["ours_checksum"]], dtype=torch.float64)
    ts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(ts, t)
    res["all_ranks_checksums"] = [float(v.item()) for v in ts]
    with open(f"{a.out}.rank{rank}.json", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
