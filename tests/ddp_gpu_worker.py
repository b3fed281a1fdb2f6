"""Multi-rank DDP worker on ONE GPU (used by tests/test_ddp_gpu.py).

RCCL refuses two ranks on one device ("Duplicate GPU detected"), so this worker
runs every rank on ``cuda:0`` with the gloo backend: the collectives go through
gloo's device-tensor path while everything else is the production GPU path --
native HIP kernels, gradients written in place into the flat buffer (grad
sinks), weight gradients on the side stream joined by the reducer before each
bucket launch, fused SGD.  Checks written to JSON:

  * DDP gradients == the average over ranks of each rank's single-process
    gradients (same weights, same per-rank batch, no DDP);
  * parameters bit-identical across ranks after a few SGD steps;
  * bucket launches in order, each once.
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_tutorials_amd import ops  # noqa: E402
from pytorch_distributed_tutorials_amd.models import build_model  # noqa: E402
from pytorch_distributed_tutorials_amd.optim import SGD  # noqa: E402
from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel, init_distributed  # noqa: E402
from pytorch_distributed_tutorials_amd.utils.seed import set_random_seeds  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--image", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--learn", type=int, default=0,
                    help="then train this many steps on a learnable set, sharded over ranks, and "
                         "record the cross-rank parameter checksums every 20 steps")
    a = ap.parse_args()
    env = init_distributed("gloo")
    rank, world = env.rank, env.world_size
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    set_random_seeds(0, deterministic=True)

    torch.manual_seed(100 + rank)  # different init per rank: DDP must broadcast rank 0's
    base = build_model(a.arch, num_classes=10, impl="native").to(dev).set_impl("native")
    ddp = DistributedDataParallel(base, bucket_cap_mb=4.0)
    # single-process twin with rank 0's weights (after the DDP broadcast)
    # (a plain module, not in a flat space: autograd returns its gradients)
    ref = build_model(a.arch, num_classes=10, impl="native").to(dev).set_impl("native")
    ref.load_state_dict(ddp.module.state_dict())

    g = torch.Generator().manual_seed(7 + rank)
    x = torch.randn(a.batch, 3, a.image, a.image, generator=g).to(dev)
    y = torch.randint(0, 10, (a.batch,), generator=g).to(dev)

    # --- gradient parity (step 1)
    opt = SGD(ddp.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    opt.zero_grad()
    ops.cross_entropy(ddp(x), y).backward()
    ref.zero_grad(set_to_none=True)
    ops.cross_entropy(ref(x), y).backward()
    torch.cuda.synchronize()
    names, mine, twin = [], [], []
    for (n, p), (_, q) in zip(ddp.module.named_parameters(), ref.named_parameters()):
        names.append(n)
        mine.append(p.grad.detach().float().reshape(-1).cpu())
        twin.append(q.grad.detach().float().reshape(-1).cpu())
    flat_twin = torch.cat(twin)
    dist.all_reduce(flat_twin)  # gloo on CPU tensors: average of the per-rank gradients
    flat_twin /= world
    flat_mine = torch.cat(mine)
    rel = ((flat_mine - flat_twin).norm() / flat_twin.norm()).item()
    per = []
    off = 0
    for n, t in zip(names, mine):
        d = flat_twin[off:off + t.numel()]
        per.append((((t - d).norm() / (d.norm() + 1e-12)).item(), n))
        off += t.numel()
    per.sort(reverse=True)
    opt.step()

    # --- a few more steps, then cross-rank equality of parameters
    for _ in range(a.steps - 1):
        opt.zero_grad()
        ops.cross_entropy(ddp(x), y).backward()
        opt.step()
    torch.cuda.synchronize()
    cs = torch.tensor([float(sum(p.detach().double().sum().item() for p in ddp.parameters()))],
                      dtype=torch.float64)
    all_cs = [torch.zeros_like(cs) for _ in range(world)]
    dist.all_gather(all_cs, cs)
    learn_cs, learn_loss = [], []
    if a.learn:
        from pytorch_distributed_tutorials_amd.data import DistributedSampler, learnable_dataset
        ds = learnable_dataset(2048, a.image, 10, device=dev, seed=5)
        sampler = DistributedSampler(len(ds), num_replicas=world, rank=rank, shuffle=True, seed=0)
        order, epoch = [], 0
        for step in range(a.learn):
            if len(order) < a.batch:
                sampler.set_epoch(epoch)
                epoch += 1
                order += list(iter(sampler))
            idx = torch.tensor(order[:a.batch], device=dev)
            order = order[a.batch:]
            opt.zero_grad()
            loss = ops.cross_entropy(ddp(ds.images[idx]), ds.labels[idx])
            loss.backward()
            opt.step()
            if step % 20 == 19 or step == a.learn - 1:
                torch.cuda.synchronize()
                c = torch.tensor([float(sum(p.detach().double().sum().item() for p in ddp.parameters()))],
                                 dtype=torch.float64)
                cs_all = [torch.zeros_like(c) for _ in range(world)]
                dist.all_gather(cs_all, c)
                learn_cs.append([float(v.item()) for v in cs_all])
                learn_loss.append(float(loss.item()))
    res = {"rank": rank, "world": world, "grad_rel_err": rel, "worst_params": per[:5],
           "learn_checksums": learn_cs, "learn_loss": learn_loss,
           "checksums": [float(c.item()) for c in all_cs],
           "launch_order": list(ddp.reducer.last_launch_order()),
           "bucket_info": ddp.bucket_info(),
           "finite": bool(torch.isfinite(flat_mine).all())}
    with open(f"{a.out}.rank{rank}.json", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
