#!/usr/bin/env python3
"""Per-workgroup phase timing of the NT conv kernel (needs a PDT_NT_TIMING variant build:
``scripts/build_variant.sh nttime -DPDT_NT_TIMING`` then ``python build/nttime/scripts/diag_nt_timing.py``).

For each conv shape: one timed launch after warm-up, then per block (s_memtime cycles)
  load  = start -> first K-step in LDS,  loop = main loop,  stats = epilogue BN statistics,
  store = bf16 staging + stores,  and per CU the blocks it ran and the idle cycles between them.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd.ops import native  # noqa: E402

SHAPES = {  # name: (C, H, W, K, R, S, stride, pad)
    "l1_conv3_64x256": (64, 56, 56, 256, 1, 1, 1, 0),
    "l1_conv1_256x64": (256, 56, 56, 64, 1, 1, 1, 0),
    "l2_conv3_128x512": (128, 28, 28, 512, 1, 1, 1, 0),
    "l2_conv1_512x128": (512, 28, 28, 128, 1, 1, 1, 0),
    "l2_3x3_128": (128, 28, 28, 128, 3, 3, 1, 1),
    "l3_conv3_256x1024": (256, 14, 14, 1024, 1, 1, 1, 0),
    "l3_conv1_1024x256": (1024, 14, 14, 256, 1, 1, 1, 0),
    "l3_3x3_256": (256, 14, 14, 256, 3, 3, 1, 1),
    "l4_3x3_512": (512, 7, 7, 512, 3, 3, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--dgrad-bn", action="store_true", help="time the BN-fused dgrad instead of the forward")
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda:0")
    N = a.batch
    print("shape, blocks, cus, kernel_us, cyc/us, load, loop, stats, store, block_total, idle_between_blocks (avg cycles)")
    for name in a.shapes.split(","):
        c, h, w, k, r, s, st, pd = SHAPES[name]
        ho, wo = (h + 2 * pd - r) // st + 1, (w + 2 * pd - s) // st + 1
        x = torch.randn(N, h, w, c, device=dev).to(torch.bfloat16)
        wt = (torch.randn(k, c, r, s, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        wk = C.pack_weight(wt, c)
        dy = torch.randn(N, ho, wo, k, device=dev).to(torch.bfloat16)
        if a.dgrad_bn:
            yb = torch.randn(N, h, w, c, device=dev).to(torch.bfloat16)
            stt = torch.stack([torch.zeros(c, device=dev), torch.ones(c, device=dev),
                               torch.ones(c, device=dev), torch.zeros(c, device=dev)])
            fn = lambda: C.conv_dgrad_bn(dy, wt, [N, h, w, c], st, pd, None, yb, None, stt, 2)  # noqa: E731
        else:
            fn = lambda: C.conv_fwd(x, wk, st, pd, True)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3
        t = C.nt_timing_fetch(8 * 65536)
        if t.numel() == 0:
            raise SystemExit("not a PDT_NT_TIMING build")
        t = t.view(-1, 8)
        valid = t[:, 4] > t[:, 0]
        # the launch's blocks: the ones stamped most recently (stale slots hold older launches)
        rt = t[:, 6]
        last = rt[valid].max()
        blk = valid & (rt > last - int(us * 100) - 200)  # realtime ticks are 10 ns
        tb = t[blk].double()
        nb = tb.shape[0]
        ph = [(tb[:, i + 1] - tb[:, i]).mean().item() for i in range(4)]
        tot = (tb[:, 4] - tb[:, 0]).mean().item()
        cu = tb[:, 7]
        # per CU: order its blocks by start, idle = start(next) - end(prev) (same CU counter)
        idle, n_idle = 0.0, 0
        for u in cu.unique():
            rows = tb[cu == u]
            rows = rows[rows[:, 0].argsort()]
            if rows.shape[0] > 1:
                d = rows[1:, 0] - rows[:-1, 4]
                idle += d.clamp(min=0).sum().item()
                n_idle += rows.shape[0] - 1
        # cycles per microsecond from the widest block's memtime/realtime ratio is not available
        # (realtime only at start); report the kernel's span in memtime over its wall time instead
        span_cyc = (tb[:, 4].max() - tb[:, 0].min()).item()
        print(f"{name}, {nb}, {cu.unique().numel()}, {us:.1f}, {span_cyc / us:.0f}, "
              + ", ".join(f"{v:.0f}" for v in ph) + f", {tot:.0f}, {idle / max(1, n_idle):.0f}", flush=True)


if __name__ == "__main__":
    main()
