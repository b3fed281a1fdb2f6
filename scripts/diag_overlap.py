#!/usr/bin/env python3
"""Does a memory-bound BN apply overlap a compute-bound conv on MI355X?

Times, for ResNet-50 (apply -> consumer conv) pairs at batch 256:
  serial : bn_act_fwd(all images) ; conv_fwd(all images)            (today's forward)
  split2 : two image halves on two streams -- apply(h1) ; [conv(h1) || apply(h2)] ; conv(h2)
so the second half's apply runs beside the first half's conv.  Prints one JSON line per pair.

    python scripts/diag_overlap.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd.ops import native  # noqa: E402

# (N, H, W, C of the applied tensor, residual?, consumer conv K, R, stride, pad)
PAIRS = [
    (256, 56, 56, 64, False, 64, 3, 1, 1),     # layer1 conv1 out -> conv2 3x3
    (256, 56, 56, 64, False, 256, 1, 1, 0),    # layer1 conv2 out -> conv3 1x1
    (256, 56, 56, 256, True, 64, 1, 1, 0),     # layer1 block out -> next conv1
    (256, 28, 28, 128, False, 512, 1, 1, 0),   # layer2 conv2 out -> conv3
    (256, 28, 28, 512, True, 128, 1, 1, 0),    # layer2 block out -> next conv1
    (256, 14, 14, 1024, True, 256, 1, 1, 0),   # layer3 block out -> next conv1
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda:0")
    s1 = torch.cuda.current_stream(dev)
    s2 = torch.cuda.Stream(dev)
    for (n, h, w, c, res, k, r, st, pd) in PAIRS:
        y = torch.randn(n, h, w, c, device=dev).to(torch.bfloat16)
        rz = torch.randn(n, h, w, c, device=dev).to(torch.bfloat16) if res else None
        sc = torch.rand(c, device=dev) + 0.5
        sh = torch.randn(c, device=dev) * 0.1
        wt = (torch.randn(k, c, r, r, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        wk = C.pack_weight(wt, c)
        hn = n // 2
        yh = (y[:hn], y[hn:])
        rh = (rz[:hn], rz[hn:]) if res else (None, None)

        def apply_only():
            C.bn_act_fwd(y, sc, sh, rz, True)

        def conv_only(z=y):
            C.conv_fwd(z, wk, st, pd, True)

        def serial():
            z = C.bn_act_fwd(y, sc, sh, rz, True)
            C.conv_fwd(z, wk, st, pd, True)

        def split2():
            z1 = C.bn_act_fwd(yh[0], sc, sh, rh[0], True)
            ev = torch.cuda.Event()
            ev.record(s1)
            s2.wait_event(ev)
            with torch.cuda.stream(s2):
                z2 = C.bn_act_fwd(yh[1], sc, sh, rh[1], True)
            C.conv_fwd(z1, wk, st, pd, True)
            with torch.cuda.stream(s2):
                C.conv_fwd(z2, wk, st, pd, True)
                ev2 = torch.cuda.Event()
                ev2.record(s2)
            s1.wait_event(ev2)
            z2.record_stream(s2)

        def split2_serial():  # same launches, one stream: isolates the launch-split cost
            z1 = C.bn_act_fwd(yh[0], sc, sh, rh[0], True)
            z2 = C.bn_act_fwd(yh[1], sc, sh, rh[1], True)
            C.conv_fwd(z1, wk, st, pd, True)
            C.conv_fwd(z2, wk, st, pd, True)

        out = {"shape": [n, h, w, c], "residual": res, "conv": [k, r, st, pd],
               "apply_ms": round(timeit(apply_only, a.iters), 4),
               "conv_ms": round(timeit(conv_only, a.iters), 4),
               "serial_ms": round(timeit(serial, a.iters), 4),
               "split2_1stream_ms": round(timeit(split2_serial, a.iters), 4),
               "split2_2stream_ms": round(timeit(split2, a.iters), 4)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
