#!/usr/bin/env python3
"""Headline benchmark: whole-node images/sec, ResNet-50 bf16 DDP training, synthetic ImageNet.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--arch resnet50] [--batch 256]
                    [--impl native|torch] [--bucket-mb 25] [--wire-dtype fp32|bf16]

For N > 1 it is launched one process per GPU by torchrun (RANK/LOCAL_RANK/
WORLD_SIZE/MASTER_* from the env); if started without torchrun and --gpus > 1
it re-launches itself through ``torch.distributed.run`` (before touching the GPU).

A timed step is the full reference training step (``resnet/main.py:119-124``):
zero_grad, forward (incl. NCHW fp32 image -> NHWC bf16), cross-entropy, backward
with bucketed gradient all-reduce over RCCL, SGD(momentum 0.9, wd 1e-5) update.
Per-GPU batch is fixed (256, the reference's per-process batch) so scaling is
weak.  W warmup steps, then exactly K steps bracketed by barrier +
synchronize; the reported time is the MAX over ranks.  ``--impl torch`` runs
the stock PyTorch-ROCm path (torch DDP + MIOpen/hipBLASLt via autocast bf16,
channels_last, foreach SGD) = the comparison baseline of BASELINE.md.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # see pytorch_distributed_tutorials_amd/__init__.py

# Stock PyTorch-ROCm ResNet-50 bf16 (bench.py --impl torch --cudnn-benchmark: MIOpen with
# solution search, hipBLASLt, autocast bf16, channels_last, foreach SGD) measured on one MI355X:
# 6634.6 img/s (38.59 ms/step, 256 img/GPU).  The reference publishes no numbers, so
# this is the number to beat.  For N > 1 the comparator is that figure x N, i.e. the stock path
# with PERFECT scaling -- an upper bound on what stock torch DDP can reach on N GPUs.
STOCK_1GPU_IMG_S = 6634.57
STOCK_BASELINE_IMG_S = {n: STOCK_1GPU_IMG_S * n for n in (1, 2, 4, 8)}


def parse(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--arch", default="resnet50")
    p.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--num-classes", type=int, default=1000)
    p.add_argument("--impl", default="native", choices=["native", "torch"])
    p.add_argument("--bucket-mb", type=float, default=25.0)
    p.add_argument("--first-bucket-mb", type=float, default=1.0,
                   help="cap of the bucket all-reduced first (torch DDP: 1 MiB)")
    p.add_argument("--last-bucket-mb", type=_last_mb, default="auto",
                   help="cap of the bucket all-reduced LAST (stem/layer1 gradients; its all-reduce "
                        "is the exposed tail): MB, 'none' (torch DDP layout) or 'auto' (default: "
                        "the xGMI tail model's choice, parallel/buckets.py auto_last_bucket_mb)")
    p.add_argument("--force-comm", action="store_true",
                   help="native impl: run the RCCL communicator + C++ reducer + buffer broadcasts "
                        "even at N=1 (world-1 RCCL communicator; exercises the multi-GPU path)")
    p.add_argument("--plan-world", type=int, default=None,
                   help="world size the bucket layout is planned for (default: the job's; with "
                        "--force-comm at N=1: 8, so one GPU runs the 8-rank layout incl. its tail bucket)")
    p.add_argument("--no-broadcast-buffers", action="store_true",
                   help="DDP broadcast_buffers=False: BatchNorm running stats stay per-rank")
    p.add_argument("--comm-timing", action="store_true",
                   help="record all-reduce time / exposed tail per step (native RCCL path)")
    p.add_argument("--deterministic", action="store_true",
                   help="deterministic kernels (slab split-K weight gradients), the trainer's default")
    p.add_argument("--wire-dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--json-out", default=None)
    p.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                   help="process-group backend for N>1 (auto: nccl = RCCL when a GPU is present)")
    p.add_argument("--share-device", action="store_true",
                   help="rehearsal only: every rank runs on cuda:0 (needs --backend gloo; RCCL "
                        "refuses two ranks on one device) so the N>1 bench path can be exercised "
                        "on a one-GPU box")
    p.add_argument("--graph", action="store_true",
                   help="capture the whole training step in a HIP graph and replay it (native impl)")
    p.add_argument("--fp8", action="store_true",
                   help="native impl: forward convs on the fp8 (e4m3) MX-rate MFMA, delayed scaling")
    p.add_argument("--watchdog-timeout", type=float, default=None,
                   help="abort a rank that makes no progress for N seconds (default 600 when N > 1, "
                        "off for one process; 0 = off): a dead peer ends the run instead of hanging it")
    p.add_argument("--comm", default="auto", choices=["auto", "rccl", "xgmi"],
                   help="gradient all-reduce backend for N>1 (native impl): RCCL (auto/rccl) or the "
                        "direct one-hop xGMI reduce-scatter/all-gather over IPC-mapped peer buffers")
    p.add_argument("--comm-timeout", type=float, default=None,
                   help="native RCCL communicator: init / per-collective timeout in seconds (600)")
    p.add_argument("--rccl-channels", default=None,
                   help="native RCCL communicator channel bounds 'min[,max]' (ncclConfig_t "
                        "minCTAs/maxCTAs; default: RCCL's choice)")
    p.add_argument("--cudnn-benchmark", action="store_true",
                   help="stock path: let MIOpen search for the fastest conv solutions")
    return p.parse_args(argv)


def _relaunch_with_torchrun(args_argv, n) -> int:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29511"),
           os.path.abspath(__file__)] + args_argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _param_checksums(ddp, impl, world, dev):
    """(all ranks identical?, rank 0's checksum): sum_i bits(p_i) * (i % 8191 + 1) in int64 over
    every parameter in order, gathered from every rank."""
    import torch
    import torch.distributed as dist
    with torch.no_grad():
        if impl == "native":
            flats = [ddp.space.param_flat]
        else:
            flats = [p.detach().reshape(-1) for p in ddp.parameters()]
        total = torch.zeros((), dtype=torch.int64, device=dev)
        base = 0
        for f in flats:
            bits = f.contiguous().view(torch.int32).to(torch.int64)
            idx = torch.arange(base, base + bits.numel(), device=bits.device, dtype=torch.int64)
            total += (bits * (idx % 8191 + 1)).sum().to(dev)
            base += bits.numel()
    if world > 1:
        if dist.get_backend() == "gloo":
            total = total.cpu()
        out = [torch.zeros_like(total) for _ in range(world)]
        dist.all_gather(out, total)
        vals = [int(v.item()) for v in out]
    else:
        vals = [int(total.item())]
    return all(v == vals[0] for v in vals), vals[0]


def _last_mb(v: str):
    if v in ("auto", "none"):
        return None if v == "none" else v
    return float(v)


def _diag_lead(step, barrier, dev, nsteps: int = 8) -> None:
    """PDT_DIAG_LEAD=1 (untimed diagnostic): how far the host's issue runs ahead of the device at
    every block forward / backward entry of ``nsteps`` back-to-back steps.  Timing events recorded at
    those points are placed on one clock with the host's perf_counter through an event recorded on
    an idle device; lead = device time the mark executed - host time it was issued (near 0: the
    device waited for the host there)."""
    import torch
    from pytorch_distributed_tutorials_amd.ops import fused
    barrier()
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    h0 = time.perf_counter()
    fused._LEAD = marks = []
    starts = []
    for _ in range(nsteps):
        starts.append(len(marks))
        fused._lead_mark("step")
        step()
    fused._LEAD = None
    barrier()
    rows = [(tag, (h - h0) * 1e3, e0.elapsed_time(ev)) for tag, h, ev in marks]
    for k, a in enumerate(starts):
        b = starts[k + 1] if k + 1 < len(starts) else len(rows)
        leads = [g - h for _, h, g in rows[a:b]]
        bw = [g - h for tag, h, g in rows[a:b] if tag.startswith("bwd")]
        print(f"[lead] step {k}: device at step start {rows[a][2]:8.2f} ms, host {rows[a][1]:8.2f} ms; "
              f"lead min {min(leads):6.2f} ms (backward min {min(bw) if bw else float('nan'):6.2f})", flush=True)
    a = starts[-1]
    for tag, h, g in rows[a:]:
        print(f"[lead]   {tag:28s} host {h:8.2f} device {g:8.2f} lead {g - h:6.2f} ms", flush=True)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _relaunch_with_torchrun(argv, args.gpus)

    import torch
    import torch.distributed as dist
    import torch.nn as nn

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pytorch_distributed_tutorials_amd import ops
    from pytorch_distributed_tutorials_amd.models import build_model
    from pytorch_distributed_tutorials_amd.optim import SGD
    from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel, init_distributed

    if args.share_device and args.backend != "gloo":
        raise SystemExit("--share-device needs --backend gloo")
    backend = args.backend if args.backend != "auto" else ("nccl" if torch.cuda.is_available() else "gloo")
    env = init_distributed(backend)
    world = env.world_size
    dev_index = 0 if args.share_device else env.local_rank
    if torch.cuda.is_available():
        torch.cuda.set_device(dev_index)
        if args.impl == "native":
            from pytorch_distributed_tutorials_amd.ops.streams import use_critical_stream
            use_critical_stream(torch.device("cuda", dev_index), collective=world > 1 or args.force_comm,
                                graph=args.graph, fp8=args.fp8)
    dev = torch.device(f"cuda:{dev_index}" if torch.cuda.is_available() else "cpu")
    dev_ids = [dev_index] if dev.type == "cuda" else None
    torch.manual_seed(0)
    if args.deterministic:
        from pytorch_distributed_tutorials_amd.utils.seed import set_random_seeds
        set_random_seeds(0, deterministic=True)

    from pytorch_distributed_tutorials_amd.utils.watchdog import Watchdog
    wd_timeout = args.watchdog_timeout if args.watchdog_timeout is not None else (600.0 if world > 1 else 0.0)
    holder = {}
    watchdog = None
    if wd_timeout > 0:
        watchdog = Watchdog(wd_timeout, rank=env.rank,
                            on_timeout=lambda: holder["ddp"].abort() if "ddp" in holder else None)
        watchdog.heartbeat("setup")

    if args.fp8:
        if args.impl != "native":
            raise SystemExit("--fp8 needs --impl native")
        ops.set_fp8(True)
    if args.impl == "native":
        from pytorch_distributed_tutorials_amd.parallel.comm import CommOptions
        copts = CommOptions.from_env(timeout=args.comm_timeout)
        if args.rccl_channels:
            ch = [int(v) for v in args.rccl_channels.split(",")]
            copts.min_channels, copts.max_channels = ch[0], ch[-1]
        model = build_model(args.arch, num_classes=args.num_classes, impl="native").to(dev)
        model.set_impl("native")
        ddp = DistributedDataParallel(model, device_ids=dev_ids, output_device=dev_ids and dev_index,
                                      bucket_cap_mb=args.bucket_mb, wire_dtype=args.wire_dtype,
                                      first_bucket_mb=args.first_bucket_mb,
                                      last_bucket_mb=args.last_bucket_mb,
                                      force_reducer=args.force_comm, comm_options=copts, comm=args.comm,
                                      broadcast_buffers=not args.no_broadcast_buffers,
                                      plan_world=args.plan_world or (8 if args.force_comm and world == 1 else None))
        holder["ddp"] = ddp
        if args.comm_timing:
            ddp.enable_comm_timing(True)
        # graph replay keeps the post-backward update: with the per-bucket update's local-mode
        # reducer attached, the replayed ResNet-18/CIFAR step ran 5.3 ms instead of 1.98 (s36)
        opt = SGD(ddp.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-5,
                  overlap=False if args.graph else None)
        criterion = ops.CrossEntropyLoss()
        autocast = None
    else:
        torch.backends.cudnn.benchmark = args.cudnn_benchmark
        model = build_model(args.arch, num_classes=args.num_classes, impl="torch").to(dev)
        model = model.to(memory_format=torch.channels_last)
        if world > 1:
            ddp = nn.parallel.DistributedDataParallel(model, device_ids=dev_ids,
                                                      output_device=dev_ids and dev_index,
                                                      bucket_cap_mb=args.bucket_mb)
        else:
            ddp = model
        opt = torch.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-5)
        criterion = nn.CrossEntropyLoss()
        autocast = torch.bfloat16

    g = torch.Generator(device="cpu").manual_seed(1234 + env.rank)
    images = torch.randn((args.batch, 3, args.image_size, args.image_size), generator=g).to(dev)
    labels = torch.randint(0, args.num_classes, (args.batch,), generator=g).to(dev)
    if args.impl == "torch":
        images = images.contiguous(memory_format=torch.channels_last)

    diag_blocked = None
    if os.environ.get("PDT_DIAG_BLOCKED") == "1" and dev.type == "cuda":
        diag_blocked = (torch.cuda.Stream(), torch.zeros(16, device=dev))

    def step():
        opt.zero_grad()
        if autocast is not None:
            with torch.autocast("cuda", dtype=autocast):
                out = ddp(images)
                loss = criterion(out, labels)
        else:
            out = ddp(images)
            loss = criterion(out, labels)
        if diag_blocked is not None:  # PDT_DIAG_BLOCKED: a side queue parked on a barrier
            ev = torch.cuda.Event()
            ev.record()
            diag_blocked[0].wait_event(ev)
            with torch.cuda.stream(diag_blocked[0]):
                diag_blocked[1].add_(1.0)
        loss.backward()
        opt.step()
        return loss

    if args.graph:
        from pytorch_distributed_tutorials_amd.utils.graph import CapturedStep
        eager_step = step
        # fp8: three graphs, one per phase of the delayed-scaling slot ring (utils/graph.py)
        from pytorch_distributed_tutorials_amd.ops.fused import FP8_RING
        step = CapturedStep(eager_step, warmup=max(1, min(args.warmup, 3)), period=3 if args.fp8 else 1,
                            ring=FP8_RING if args.fp8 else None)

    def barrier():
        if world > 1:
            dist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def beat(phase):
        if watchdog is not None:
            watchdog.heartbeat(phase)

    for i in range(args.warmup):
        beat(f"warmup {i}")
        loss = step()
    beat("barrier")
    barrier()
    t0 = time.perf_counter()
    host = 0.0  # host time spent inside step() (issue time; ~= step time when the host is the bound)
    for i in range(args.steps):
        beat(f"step {i}")
        th = time.perf_counter()
        loss = step()
        host += time.perf_counter() - th
    barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    final_loss = float(loss.item())
    # host issue cost of one step from an idle device (untimed, after the timed region): the time
    # inside step() above also counts waits on a full launch queue whenever the GPU is the bound
    issue = []
    prof_path = os.environ.get("PDT_HOST_PROFILE")  # cProfile of these idle-device steps (diagnostic)
    prof = None
    if prof_path and env.rank == 0:
        import cProfile
        prof = cProfile.Profile()
    for _ in range(3):
        barrier()
        th = time.perf_counter()
        if prof is not None:
            # backward on this thread, so cProfile sees the autograd Functions' Python too
            with torch.autograd.set_multithreading_enabled(False):
                prof.enable()
                step()
                prof.disable()
        else:
            step()
        issue.append(time.perf_counter() - th)
    barrier()
    if prof is not None:
        import io
        import pstats
        buf = io.StringIO()
        st_ = pstats.Stats(prof, stream=buf)
        st_.sort_stats("tottime").print_stats(60)
        st_.sort_stats("cumulative").print_stats(60)
        with open(prof_path, "w") as f:
            f.write(buf.getvalue())
    host_issue_ms = 1000.0 * min(issue)
    if os.environ.get("PDT_DIAG_LEAD") == "1" and dev.type == "cuda" and args.impl == "native":
        _diag_lead(step, barrier, dev)
    # every rank must hold bit-identical parameters after the run (untimed): a positional int64
    # checksum of the parameter bits, all-gathered -- a fast-but-wrong multi-GPU run shows here
    ranks_identical, param_checksum = _param_checksums(ddp, args.impl, world, dev)
    comm = None
    if args.impl == "native":
        info = ddp.bucket_info()
        comm = {"native_comm": info["native_comm"], "reducer": info["reducer"], "xgmi": info["xgmi"], "wgrad_cu_reserve": info.get("wgrad_cu_reserve", 0),
                "buckets_mb": [round(b / 2**20, 2) for b in info["bucket_bytes"]]}
        # diagnostics for the scaling run (untimed, after the timed region): what the communicator
        # reports about itself, and one step's all-reduce time / exposed tail from the reducer's
        # HIP events (time from the first bucket's launch to the last bucket's end on the comm
        # stream; exposed = the part after the backward's last kernel)
        comm.update(ddp.comm_diagnostics())
        if not args.comm_timing and not args.graph and ddp.enable_comm_timing(True):
            step()
            barrier()
        st = ddp.comm_stats()
        if st is not None:
            comm["comm_ms"] = round(st["comm_ms"], 3)
            comm["exposed_ms"] = round(st["exposed_ms"], 3)
            comm["last_step"] = st
        if not comm["count_matches_world"] and env.rank == 0:
            print(f"[bench] WARNING: the communicator reports {comm['comm_count']} ranks but WORLD_SIZE is "
                  f"{world}: collectives do not span the job", flush=True)

    if env.rank == 0:
        img_s = world * args.batch * args.steps / elapsed
        base = STOCK_BASELINE_IMG_S.get(world) if args.arch == "resnet50" else None
        res = {
            "metric": "images/sec (whole node) ResNet-50 bf16 at 1/2/4/8 MI355X"
            if args.arch == "resnet50" and not args.fp8
            else f"images/sec (whole node) {args.arch} {'fp8' if args.fp8 else 'bf16'}",
            "value": round(img_s, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "host_ms_per_step": round(1000.0 * host / args.steps, 3),
            "host_issue_ms": round(host_issue_ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(img_s / base, 4) if base else None),
            "dtype": "fp8" if args.fp8 else "bf16",
            "data": f"synthetic (ImageNet-shaped 3x{args.image_size}x{args.image_size} fp32 images, random labels, "
                    "random-init weights)",
            "config": {"model": args.arch, "global_batch": args.batch * world,
                       "seq_len": None, "image_size": args.image_size,
                       "parallelism": f"dp{world}", "impl": args.impl,
                       "backend": backend, "shared_device": bool(args.share_device),
                       "bucket_mb": args.bucket_mb, "wire_dtype": args.wire_dtype, "comm_backend": args.comm,
                       "cudnn_benchmark": bool(args.cudnn_benchmark), "graph": bool(args.graph),
                       "deterministic": bool(args.deterministic), "force_comm": bool(args.force_comm),
                       "first_bucket_mb": args.first_bucket_mb,
                       "last_bucket_mb": ddp.last_bucket_mb if args.impl == "native" else args.last_bucket_mb,
                       "plan_world": getattr(ddp, "plan_world", world) if args.impl == "native" else world,
                       "comm": comm, "final_loss": round(final_loss, 4),
                       "ranks_identical": ranks_identical, "param_checksum": param_checksum},
        }
        line = json.dumps(res)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if watchdog is not None:
        watchdog.stop()
    if world > 1:
        barrier()
        dist.destroy_process_group()
        # every rank is past its last collective: end the process here rather than in interpreter
        # teardown, where the native communicator's destructor would run in an unspecified order
        # with torch's (a late peer must not be able to hold a finished rank at exit)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
