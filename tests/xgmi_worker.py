"""Worker for tests/test_xgmi_gpu.py: the direct xGMI all-reduce between PROCESSES.

All ranks share cuda:0 (same-device IPC: the one-GPU box has no peers), gloo process group for
the rendezvous and the reference all-reduce.  Modes:

* ``buckets``: each rank fills the shared gradient buffer with its own random data, all-reduces a
  few buckets (aligned float4 path and odd-offset scalar path, two epochs each) through
  ``XgmiComm`` and compares with gloo's all-reduce of the same fp32 data (bitwise at world 2) and
  with the rank-order fp32 sum (bitwise at any world);
* ``ddp``: ResNet-18 (native kernels) under ``DistributedDataParallel(comm="xgmi")`` vs the same
  model under the gloo-reduced DDP, one step from identical weights/data: gradients bitwise.

Prints one RESULT json line per rank.  A runtime that refuses same-device IPC reports
``ipc_refused`` with the exact error instead of failing.
"""
import argparse
import json
import os
import sys
import traceback

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_tutorials_amd.parallel import init_distributed  # noqa: E402


def run_buckets(rank, world, dev):
    from pytorch_distributed_tutorials_amd.parallel.xgmi import xgmi_comm
    n = 1 << 20
    buckets = [(0, 400000), (400000, 300001), (700001, 348575)]  # aligned, odd count, odd offset
    comm = xgmi_comm(dev, n, len(buckets), timeout=60.0)
    g = comm.grad_buffer()
    res = {"bitwise_vs_rank_order": True, "bitwise_vs_gloo": True, "max_abs_vs_gloo": 0.0}
    for epoch in range(2):
        gen = torch.Generator().manual_seed(1000 * epoch + rank)
        mine = torch.randn(n, generator=gen)
        g.copy_(mine.to(dev))
        torch.cuda.synchronize()
        for b, (off, cnt) in enumerate(buckets):
            comm.reduce_bucket(b, off, cnt, True)
        comm.synchronize()
        got = g.cpu()
        # references: gloo all-reduce of the same fp32 data / world, and the rank-order sum
        ref = mine.clone()
        dist.all_reduce(ref)
        ref /= world
        alls = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(alls, mine)
        ordered = alls[0].clone()
        for q in range(1, world):
            ordered += alls[q]
        ordered /= world
        covered = torch.zeros(n, dtype=torch.bool)
        for off, cnt in buckets:
            covered[off:off + cnt] = True
        res["bitwise_vs_rank_order"] &= bool(torch.equal(got[covered], ordered[covered]))
        res["bitwise_vs_gloo"] &= bool(torch.equal(got[covered], ref[covered]))
        res["max_abs_vs_gloo"] = max(res["max_abs_vs_gloo"], float((got - ref)[covered].abs().max()))
        res["untouched_kept"] = bool(torch.equal(got[~covered], mine[~covered])) if (~covered).any() else True
    res["error_code"] = comm.error_code
    return res


def run_ddp(rank, world, dev):
    import copy
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel
    from pytorch_distributed_tutorials_amd.utils.seed import set_random_seeds
    set_random_seeds(0, deterministic=True)  # slab split-K weight gradients: bitwise repeatable
    torch.manual_seed(0)
    base = build_model("resnet18", num_classes=10).to(dev)
    gen = torch.Generator().manual_seed(50 + rank)
    x = torch.randn(8, 3, 32, 32, generator=gen).to(dev)
    y = torch.randint(0, 10, (8,), generator=gen).to(dev)
    grads = {}
    for mode in ("gloo", "xgmi"):
        m = copy.deepcopy(base).set_impl("native")
        ddp = DistributedDataParallel(m, device_ids=[dev.index], comm="xgmi" if mode == "xgmi" else "auto")
        loss = ops.cross_entropy(ddp(x), y)
        loss.backward()
        torch.cuda.synchronize()
        grads[mode] = ddp.space.grad_flat.detach().cpu().clone()
        info = ddp.bucket_info()
        if mode == "xgmi":
            assert info["xgmi"] and info["num_buckets"] >= 1, info
    return {"ddp_bitwise": bool(torch.equal(grads["gloo"], grads["xgmi"])),
            "ddp_max_abs": float((grads["gloo"] - grads["xgmi"]).abs().max()),
            "grad_norm": float(grads["xgmi"].norm())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="buckets", choices=["buckets", "ddp"])
    a = ap.parse_args()
    env = init_distributed("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    out = {"rank": env.rank, "world": env.world_size}
    try:
        out.update(run_buckets(env.rank, env.world_size, dev) if a.mode == "buckets" else
                   run_ddp(env.rank, env.world_size, dev))
        out["status"] = "ok"
    except RuntimeError as e:
        msg = str(e)
        out["status"] = "ipc_refused" if "hipIpc" in msg else "error"
        out["error"] = msg
        out["trace"] = traceback.format_exc()[-2000:]
    print("RESULT " + json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if out["status"] in ("ok", "ipc_refused") else 1


if __name__ == "__main__":
    raise SystemExit(main())
