import sys
import torch
sys.path.insert(0, ".")
torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
from pytorch_distributed_tutorials_amd.ops._ext import native  # noqa: E402
from pytorch_distributed_tutorials_amd.ops import reference as ref  # noqa: E402
C = native()
dev = torch.device("cuda:0")
for (n, h, c, k, r, st, pd) in [(32, 8, 64, 64, 3, 1, 1), (32, 16, 64, 64, 3, 1, 1), (32, 8, 64, 128, 3, 1, 1),
                                (4, 56, 64, 64, 3, 1, 1), (32, 8, 128, 64, 1, 1, 0), (8, 8, 64, 64, 3, 1, 1)]:
    x = torch.randn(n, h, h, c, device=dev).bfloat16()
    ho = (h + 2 * pd - r) // st + 1
    dy = torch.randn(n, ho, ho, k, device=dev).bfloat16()
    ref_dw = ref.conv2d_nhwc_wgrad(dy.float(), x.float(), (k, c, r, r), st, pd)
    for det in (True, False):
        dw = C.conv_wgrad(dy, x, [k, c, r, r], st, pd, det)
        sink = torch.zeros(k, c, r, r, device=dev).contiguous(memory_format=torch.channels_last)
        C.conv_wgrad(dy, x, [k, c, r, r], st, pd, det, sink)
        torch.cuda.synchronize()
        e1 = ((dw.float() - ref_dw).norm() / ref_dw.norm()).item()
        e2 = ((sink - ref_dw).norm() / ref_dw.norm()).item()
        print(f"n{n} h{h} c{c} k{k} r{r} det={det}: out nan {int(torch.isnan(dw).sum())} err {e1:.2e} | "
              f"sink nan {int(torch.isnan(sink).sum())} err {e2:.2e}", flush=True)
