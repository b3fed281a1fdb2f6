#!/usr/bin/env python3
"""Per-parameter gradient agreement of the native bf16 ResNet against the fp32 stock model, with
stock autocast-bf16 as the noise yardstick (same weights, same batch).

    python scripts/diag_parity.py [--arch resnet50] [--batch 32] [--size 112]
"""
import argparse
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd import ops  # noqa: E402
from pytorch_distributed_tutorials_amd.models import build_model  # noqa: E402


def grads(m):
    return {n: p.grad.float().flatten().clone() for n, p in m.named_parameters()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=112)
    ap.add_argument("--eval", action="store_true", help="BN in eval mode (running stats)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    mt = build_model(a.arch, num_classes=1000).to(dev)
    mb = copy.deepcopy(mt)
    mn = copy.deepcopy(mt).set_impl("native")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(a.batch, 3, a.size, a.size, generator=g).to(dev)
    y = torch.randint(0, 1000, (a.batch,), generator=g).to(dev)
    if a.eval:
        for m in (mt, mb, mn):
            m.eval()
    lt = F.cross_entropy(mt(x), y)
    lt.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lb = F.cross_entropy(mb(x), y)
    lb.backward()
    ln = ops.cross_entropy(mn(x), y)
    ln.backward()
    print(f"loss fp32 {lt.item():.5f} autocast-bf16 {lb.item():.5f} native {ln.item():.5f}")
    gt, gb, gn = grads(mt), grads(mb), grads(mn)
    cos = lambda u, v: F.cosine_similarity(u, v, dim=0).item()  # noqa: E731
    print(f"{'param':40s} {'|g| fp32':>10s} {'|g| nat':>10s} {'cos(nat)':>9s} {'cos(bf16)':>9s}")
    for n in gt:
        print(f"{n:40s} {gt[n].norm():10.3e} {gn[n].norm():10.3e} {cos(gn[n], gt[n]):9.4f} {cos(gb[n], gt[n]):9.4f}")
    cat = lambda d: torch.cat(list(d.values()))  # noqa: E731
    print(f"GLOBAL cos native {cos(cat(gn), cat(gt)):.4f}  autocast-bf16 {cos(cat(gb), cat(gt)):.4f}")


if __name__ == "__main__":
    main()
