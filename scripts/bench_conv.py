#!/usr/bin/env python3
"""Per-shape conv microbenchmark: native implicit-GEMM kernels vs stock MIOpen (torch).

    python scripts/bench_conv.py [--arch resnet50] [--batch 256] [--iters 10] [--torch]

Enumerates every distinct conv of the model at the given batch (with its repeat
count), times fwd / dgrad / wgrad of the native kernels (and optionally torch's
bf16 channels_last conv through MIOpen), and prints ms, TFLOP/s and the
count-weighted share of the whole network, as CSV-like rows + a JSON summary.
"""
import argparse
import json
import os
import sys
from collections import OrderedDict

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd.models import build_model  # noqa: E402
from pytorch_distributed_tutorials_amd.ops import native  # noqa: E402


def conv_shapes(arch, batch, image):
    m = build_model(arch)
    shapes = OrderedDict()
    hooks = []

    def hook(mod, inp, out):
        x = inp[0]
        key = (x.shape[1], x.shape[2], x.shape[3], mod.out_channels, mod.kernel_size[0],
               mod.kernel_size[1], mod.stride[0], mod.padding[0])
        shapes[key] = shapes.get(key, 0) + 1
    for mod in m.modules():
        if isinstance(mod, nn.Conv2d):
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m(torch.zeros(1, 3, image, image))
    return shapes


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--torch", action="store_true", help="also time MIOpen via torch")
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="single shape CxHxWxKxRxSxstridexpad")
    ap.add_argument("--fp8", action="store_true", help="also time the fp8 (e4m3) forward conv")
    ap.add_argument("--bn", action="store_true", help="also time dgrad with the fused BN-backward epilogue")
    ap.add_argument("--det", action="store_true", help="wgrad in deterministic mode (split-K slabs + reduce)")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad", help="which products to time (others report 0)")
    ap.add_argument("--force", default=None,
                    help="NT tile-policy test hook 'k32/mid/wide' (-1 policy, 0 off, 1 on): C.conv_nt_force")
    a = ap.parse_args()
    C = native()
    if a.force:
        C.conv_nt_force(*[int(v) for v in a.force.split("/")])
    dev = torch.device("cuda:0")
    N = a.batch
    rows = []
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "t_fwd": 0.0, "t_dgrad": 0.0, "t_wgrad": 0.0, "flop": 0.0}
    print("C,H,W,K,R,S,st,pd,count,M,N,K_gemm,fwd_ms,fwd_TF,dgrad_ms,dgrad_TF,wgrad_ms,wgrad_TF"
          + (",torch_fwd_ms,torch_dgrad_ms,torch_wgrad_ms" if a.torch else "")
          + (",fp8_fwd_ms,fp8_fwd_TF" if a.fp8 else "")
          + (",dgrad_bn_ms" if a.bn else ""))
    tot["dgrad_bn"] = 0.0
    tot["f8_fwd"] = 0.0
    shapes = conv_shapes(a.arch, N, a.image)
    if a.only:
        want = tuple(int(v) for v in a.only.split("x"))
        shapes = OrderedDict([(want, 1)])
    for (c, h, w, k, r, s, st, pd), cnt in shapes.items():
        cx = c if c % 8 == 0 else 8
        ho = (h + 2 * pd - r) // st + 1
        wo = (w + 2 * pd - s) // st + 1
        x = torch.randn(N, h, w, cx, device=dev).to(torch.bfloat16)
        wt = (torch.randn(k, c, r, s, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        wk = C.pack_weight(wt, cx)
        dy = torch.randn(N, ho, wo, k, device=dev).to(torch.bfloat16)
        flop = 2.0 * N * ho * wo * k * c * r * s
        ops = a.ops.replace("+", ",").split(",")
        f = timeit(lambda: C.conv_fwd(x, wk, st, pd, True), a.iters) if "fwd" in ops else 0.0
        d = timeit(lambda: C.conv_dgrad(dy, wt, [N, h, w, c], st, pd), a.iters) \
            if c % 8 == 0 and "dgrad" in ops else 0.0
        g = timeit(lambda: C.conv_wgrad(dy, x, [k, c, r, s], st, pd, a.det), a.iters) if "wgrad" in ops else 0.0
        row = [c, h, w, k, r, s, st, pd, cnt, N * ho * wo, k, c * r * s,
               round(f, 3), round(flop / f / 1e9, 1) if f else 0, round(d, 3), round(flop / d / 1e9, 1) if d else 0,
               round(g, 3), round(flop / g / 1e9, 1) if g else 0]
        tot["fwd"] += f * cnt
        tot["dgrad"] += d * cnt
        tot["wgrad"] += g * cnt
        tot["flop"] += flop * cnt
        if a.torch:
            xt = x[..., :c].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            wtb = wt.to(torch.bfloat16).requires_grad_(True)
            dyt = dy.permute(0, 3, 1, 2)
            tf = timeit(lambda: torch.nn.functional.conv2d(xt, wtb, stride=st, padding=pd), a.iters)
            td = timeit(lambda: torch.ops.aten.convolution_backward(
                dyt, xt, wtb, None, (st, st), (pd, pd), (1, 1), False, (0, 0), 1, (True, False, False)), a.iters)
            tw = timeit(lambda: torch.ops.aten.convolution_backward(
                dyt, xt, wtb, None, (st, st), (pd, pd), (1, 1), False, (0, 0), 1, (False, True, False)), a.iters)
            row += [round(tf, 3), round(td, 3), round(tw, 3)]
            tot["t_fwd"] += tf * cnt
            tot["t_dgrad"] += td * cnt
            tot["t_wgrad"] += tw * cnt
        if a.fp8:
            if cx % 16 == 0:
                st8 = torch.zeros(C.fp8_state_floats(), device=dev)
                x8 = C.quant_e4m3(x, st8, 0)
                d0 = C.fp8_deq_offset()
                wq, osc = C.pack_weight_fp8(wt, cx, st8[d0:d0 + 1])
                f8 = timeit(lambda: C.conv_fwd_fp8(x8, wq, osc, st, pd, True), a.iters)
            else:
                f8 = f
            row += [round(f8, 3), round(flop / f8 / 1e9, 1)]
            tot["f8_fwd"] += f8 * cnt
        if a.bn:
            if c % 8 == 0:
                yb = torch.randn(N, h, w, c, device=dev).to(torch.bfloat16)
                stt = torch.stack([torch.zeros(c, device=dev), torch.ones(c, device=dev),
                                   torch.ones(c, device=dev), torch.zeros(c, device=dev)])
                db = timeit(lambda: C.conv_dgrad_bn(dy, wt, [N, h, w, c], st, pd, None, yb, None, stt, 2),
                            a.iters)
            else:
                db = 0.0
            row += [round(db, 3)]
            tot["dgrad_bn"] += db * cnt
        print(",".join(str(v) for v in row), flush=True)
        rows.append(row)
    summ = {k: round(v, 3) for k, v in tot.items() if k != "flop"}
    allms = tot["fwd"] + tot["dgrad"] + tot["wgrad"]
    summ["native_total_ms"] = round(allms, 3)
    summ["native_TFLOPs"] = round(3 * tot["flop"] / allms / 1e9, 1) if allms else 0
    print(json.dumps(summ))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"rows": rows, "summary": summ}, fh)


if __name__ == "__main__":
    main()
