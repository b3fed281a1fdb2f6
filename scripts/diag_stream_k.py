"""Stream-K NT diagnostics: run one conv shape several times (and with fresh inputs in between)
and report where repeated outputs / BN partials differ.  PDT_NT_SK selects the mode.

    PDT_NT_SK=1 python scripts/diag_stream_k.py 256 7 7 512 512 3
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_tutorials_amd import _C as C  # noqa: E402
from pytorch_distributed_tutorials_amd.ops import reference as ref  # noqa: E402

n, h, w, c, k, r = (int(v) for v in sys.argv[1:7])
pd = r // 2
dev = torch.device("cuda:0")


def operands(seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, h, w, c, generator=g).to(torch.bfloat16).to(dev)
    wt = (torch.randn(k, c, r, r, generator=g) / (c * r * r) ** 0.5).to(torch.bfloat16).float().to(dev)
    return x, wt.contiguous(memory_format=torch.channels_last)


x, wt = operands(1)
x2, wt2 = operands(2)
pk, pk2 = C.pack_weight(wt, c), C.pack_weight(wt2, c)
runs = []
for i in range(4):
    y, p = C.conv_fwd(x, pk, 1, pd, True)
    y3, p3 = C.conv_fwd(x2, pk2, 1, pd, True)  # different data in between
    torch.cuda.synchronize()
    runs.append((y.clone(), p.clone()))
yr = ref.conv2d_nhwc(x, wt, 1, pd)
yr3 = ref.conv2d_nhwc(x2, wt2, 1, pd)
rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
out = {"sk_launches": C.conv_stream_k_launches(), "rel": [rel(y, yr) for y, _ in runs], "rel_other": rel(y3, yr3)}
y0, p0 = runs[0]
for i, (y, p) in enumerate(runs[1:], 1):
    dy = (y.float() - y0.float()).abs()
    bad = (dy > 0).reshape(-1, k)  # [M][Nout]
    rows = bad.any(1).nonzero().flatten()
    cols = bad.any(0).nonzero().flatten()
    out[f"run{i}"] = {"y_equal": bool(torch.equal(y, y0)), "p_equal": bool(torch.equal(p, p0)),
                      "y_maxdiff": dy.max().item(), "bad_rows": rows.numel(),
                      "row_tiles": sorted(set((rows // 256).tolist()))[:20],
                      "col_tiles": sorted(set((cols // 256).tolist())),
                      "p_rows_bad": ((p - p0).abs().reshape(p.shape[0], -1) > 0).any(1).nonzero().flatten().tolist()[:20]}
print(json.dumps(out))
