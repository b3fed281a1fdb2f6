"""Locate the first native op whose outputs contain NaN when uninitialised memory is NaN-filled."""
import copy
import os
import sys

import torch

sys.path.insert(0, ".")
torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
from pytorch_distributed_tutorials_amd.ops import _ext  # noqa: E402

real = _ext.native()
seen = {"first": None, "count": 0}


def has_nan(o):
    if isinstance(o, torch.Tensor):
        return o.is_floating_point() and bool(torch.isnan(o).any())
    if isinstance(o, (tuple, list)):
        return any(has_nan(t) for t in o)
    return False


def desc(o):
    if isinstance(o, torch.Tensor):
        return f"{tuple(o.shape)}:{o.dtype}"
    if isinstance(o, (tuple, list)):
        return "(" + ",".join(desc(t) for t in o) + ")"
    return type(o).__name__


log = []  # (op name, arg descriptions, output references)
SYNC = os.environ.get("OP_SYNC", "0") == "1"


class Proxy:
    def __getattr__(self, name):
        f = getattr(real, name)
        if not callable(f) or isinstance(f, type):
            return f

        def wrapped(*a, **k):
            out = f(*a, **k)
            if SYNC:
                torch.cuda.synchronize()
            if name not in ("pack_t_batched", "cast_to_bf16", "sgd_step"):
                log.append((name, [desc(v) for v in a], out,
                            [v for v in a if isinstance(v, torch.Tensor)]))
            return out
        return wrapped


def report(tag):
    torch.cuda.synchronize()
    for i, (name, ins, out, args) in enumerate(log):
        if has_nan(out):
            bad_in = [j for j, v in enumerate(args) if has_nan(v)]
            print(f"[{tag}] first op with NaN output: #{i} {name} args {ins} nan-input-tensors {bad_in} "
                  f"out {desc(out)}", flush=True)
            break
    else:
        print(f"[{tag}] no NaN outputs in {len(log)} ops", flush=True)
    log.clear()


proxy = Proxy()
_ext.native = lambda: proxy
import pytorch_distributed_tutorials_amd.ops.fused as fused  # noqa: E402
fused.native = lambda: proxy
import pytorch_distributed_tutorials_amd.optim.sgd as sgdmod  # noqa: E402
sgdmod.native = lambda: proxy

from pytorch_distributed_tutorials_amd import ops  # noqa: E402
from pytorch_distributed_tutorials_amd.models import build_model  # noqa: E402
from pytorch_distributed_tutorials_amd.optim import SGD  # noqa: E402
from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = build_model(os.environ.get("ARCH", "resnet18"), num_classes=10).to(dev).set_impl("native")
ddp = DistributedDataParallel(m)
opt = SGD(ddp.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
x = torch.randn(32, 3, 32, 32, device=dev)
y = torch.randint(0, 10, (32,), device=dev)
for it in range(2):
    opt.zero_grad()
    loss = ops.cross_entropy(ddp(x), y)
    loss.backward()
    report(f"step{it}")
    print("loss", float(loss.detach()), flush=True)
    opt.step()
    torch.cuda.synchronize()
    log.clear()
