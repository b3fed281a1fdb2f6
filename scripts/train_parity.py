#!/usr/bin/env python3
"""Training-level parity: the native bf16 path vs the stock fp32 path, same init, same data.

Trains ResNet-18 (the reference model, resnet/main.py:76; ``--arch resnet50 --image 112`` for the
headline model) on a learnable synthetic CIFAR-shaped set (class templates + noise, ``data.learnable_dataset``) with the reference optimizer
(SGD lr 0.01, momentum 0.9, wd 1e-5, resnet/main.py:103) for ``--steps`` steps:

* native: our NHWC bf16 kernels, our DDP wrapper (world 1: flat buffers, in-place gradient
  sinks), fused SGD;
* stock:  the same weights as a plain fp32 torch model (impl="torch") with torch.optim.SGD.

Both see identical batches (one fixed permutation per epoch).  Prints one JSON line with the
per-window mean losses of both runs and the final train accuracy (eval mode, whole set).

    python scripts/train_parity.py [--steps 200] [--batch 128] [--json out.json]
"""
import argparse
import copy
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd import ops  # noqa: E402
from pytorch_distributed_tutorials_amd.data import learnable_dataset  # noqa: E402
from pytorch_distributed_tutorials_amd.models import build_model  # noqa: E402
from pytorch_distributed_tutorials_amd.optim import SGD  # noqa: E402
from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel  # noqa: E402


def accuracy(model, ds, native, bs=500):
    model.eval()
    correct = 0
    with torch.no_grad():
        for i in range(0, len(ds), bs):
            x, y = ds.images[i:i + bs], ds.labels[i:i + bs]
            out = model(x)
            correct += int((ops.top1_correct(out, y) if native else (out.argmax(1) == y).sum()).item())
    model.train()
    return correct / len(ds)


def main():
    # stock convolutions through PyTorch's own im2col + BLAS path, not MIOpen: on a fresh box MIOpen
    # compiles every conv shape first (minutes, silently), and the fp32 reference needs no MIOpen
    torch.backends.cudnn.enabled = False
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--samples", type=int, default=4096)
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--window", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--image", type=int, default=32, help="image side (32: CIFAR-shaped)")
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--fp8", action="store_true",
                    help="native side on the fp8 path (e4m3 activations / e5m2 gradients, fp8 wgrad)")
    ap.add_argument("--fp8-parts", default="all", choices=["all", "fwd", "fwd+dgrad"],
                    help="diagnostics: which GEMMs take fp8 (forward only / + input gradients / + weight "
                         "gradients)")
    ap.add_argument("--deterministic", action="store_true",
                    help="native side in deterministic mode (the reference's cudnn.deterministic=True: "
                         "fixed-order reductions, slab split-K weight gradients): one run is reproducible "
                         "bit for bit, so a single-run criterion tests the trajectory, not one draw of noise")
    ap.add_argument("--repeats", type=int, default=1,
                    help="native runs from the same init and data order (stock runs once); the JSON's "
                         "native curve is their mean, the single runs are listed too")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.deterministic:
        from pytorch_distributed_tutorials_amd.utils.seed import set_random_seeds
        set_random_seeds(0, deterministic=True)
        torch.backends.cudnn.enabled = False  # (set_random_seeds flips cudnn flags; keep MIOpen off)
    if a.fp8:
        ops.set_fp8(True)
        from pytorch_distributed_tutorials_amd.ops import fused
        fused._FP8_BWD = a.fp8_parts != "fwd"
        fused._FP8_WGRAD = a.fp8_parts == "all"
        fused._FP8_ONLY = a.fp8_parts == "all" 
    ds = learnable_dataset(a.samples, a.image, a.classes, device=dev, seed=3, noise=a.noise)
    torch.manual_seed(0)
    stock = build_model(a.arch, num_classes=a.classes).to(dev)
    init = copy.deepcopy(stock)

    def batches():
        g = torch.Generator().manual_seed(11)
        perm = torch.randperm(len(ds), generator=g).to(dev)
        pos = 0
        for _ in range(a.steps):
            if pos + a.batch > len(ds):
                perm = torch.randperm(len(ds), generator=g).to(dev)
                pos = 0
            idx = perm[pos:pos + a.batch]
            pos += a.batch
            yield ds.images[idx], ds.labels[idx]

    runs, accs = [], []
    for _ in range(a.repeats):
        native_m = copy.deepcopy(init).set_impl("native")
        native = DistributedDataParallel(native_m)          # world 1: flat space + grad sinks
        opt_n = SGD(native.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-5)
        ln = []
        for x, y in batches():
            opt_n.zero_grad()
            loss_n = ops.cross_entropy(native(x), y)
            loss_n.backward()
            opt_n.step()
            ln.append(loss_n.detach())
        runs.append(torch.stack(ln).float().cpu())
        accs.append(accuracy(native, ds, True))
        del native, native_m, opt_n
    opt_s = torch.optim.SGD(stock.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-5)
    ls = []
    for x, y in batches():
        opt_s.zero_grad()
        loss_s = F.cross_entropy(stock(x), y)
        loss_s.backward()
        opt_s.step()
        ls.append(loss_s.detach())
    ln = torch.stack(runs).mean(0)
    ls = torch.stack(ls).float().cpu()
    w = a.window
    nwin = a.steps // w
    res = {
        "arch": a.arch, "image": a.image, "fp8": bool(a.fp8), "fp8_parts": a.fp8_parts if a.fp8 else None,
        "steps": a.steps, "batch": a.batch, "samples": a.samples, "noise": a.noise, "lr": a.lr,
        "window": w,
        "native_window_loss": [round(float(ln[i * w:(i + 1) * w].mean()), 4) for i in range(nwin)],
        "stock_window_loss": [round(float(ls[i * w:(i + 1) * w].mean()), 4) for i in range(nwin)],
        "native_train_acc": min(accs),
        "native_train_accs": accs,
        "native_window_loss_runs": [[round(float(r[i * w:(i + 1) * w].mean()), 4) for i in range(nwin)]
                                    for r in runs],
        "stock_train_acc": accuracy(stock, ds, False),
        "finite": bool(all(torch.isfinite(r).all() for r in runs) and torch.isfinite(ls).all()),
        "repeats": a.repeats,
        "deterministic": bool(a.deterministic),
    }
    line = json.dumps(res)
    print(line, flush=True)
    if a.json:
        with open(a.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
