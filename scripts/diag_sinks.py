"""Diagnostic: gradient agreement between plain-autograd and flat-sink (DDP) paths, with the
wgrad side stream on/off and deterministic on/off; also run-to-run variation of each path."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from pytorch_distributed_tutorials_amd import ops  # noqa: E402
from pytorch_distributed_tutorials_amd.models import build_model  # noqa: E402
from pytorch_distributed_tutorials_amd.ops import streams  # noqa: E402
from pytorch_distributed_tutorials_amd.parallel import DistributedDataParallel  # noqa: E402
from pytorch_distributed_tutorials_amd.utils import seed as seedmod  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def grads(model, wrap, x, y, iters=2):
    for p in model.parameters():
        p.grad = None
    m = DistributedDataParallel(model) if wrap else model
    for _ in range(iters):
        ops.cross_entropy(m(x), y).backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().clone() for n, p in model.named_parameters()}


dev = torch.device("cuda:0")
torch.manual_seed(0)
base = build_model("resnet50", num_classes=10).to(dev).set_impl("native")
x = torch.randn(2, 3, 64, 64, device=dev)
y = torch.randint(0, 10, (2,), device=dev)
for det in (True, False):
    seedmod._DETERMINISTIC = det
    for side in (False, True):
        streams.set_enabled(side)
        g_plain = grads(copy.deepcopy(base), False, x, y)
        g_plain2 = grads(copy.deepcopy(base), False, x, y)
        g_flat = grads(copy.deepcopy(base), True, x, y)
        g_flat2 = grads(copy.deepcopy(base), True, x, y)
        worst = sorted(((rel(g_flat[n], g_plain[n]), n) for n in g_plain), reverse=True)[:4]
        print(f"det={det} side={side} plain-vs-plain {max(rel(g_plain2[n], g_plain[n]) for n in g_plain):.2e} "
              f"flat-vs-flat {max(rel(g_flat2[n], g_flat[n]) for n in g_plain):.2e} "
              f"flat-vs-plain worst {[(round(e, 4), n) for e, n in worst]}", flush=True)
