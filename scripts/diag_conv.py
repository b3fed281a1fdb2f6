import sys
import torch
sys.path.insert(0, ".")
torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
from pytorch_distributed_tutorials_amd.ops._ext import native  # noqa: E402
C = native()
dev = torch.device("cuda:0")
for (n, h, c, k, r, st, pd) in [(32, 8, 64, 64, 3, 1, 1), (32, 8, 64, 64, 1, 1, 0), (32, 16, 64, 64, 3, 1, 1),
                                (4, 56, 64, 64, 3, 1, 1), (32, 8, 64, 128, 3, 2, 1), (32, 4, 128, 128, 3, 1, 1)]:
    x = torch.randn(n, h, h, c, device=dev).bfloat16()
    w = (torch.randn(k, c, r, r, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    wk = C.pack_weight(w, c)
    y, part = C.conv_fwd(x, wk, st, pd, True)
    torch.cuda.synchronize()
    ny = torch.isnan(y.float())
    npart = torch.isnan(part)
    rows = ny.reshape(-1, k).any(1).nonzero().flatten()
    print(f"n{n} h{h} c{c} k{k} r{r} s{st}: y NaN {int(ny.sum())}/{y.numel()} rows {rows[:8].tolist()}.. "
          f"part {tuple(part.shape)} NaN {int(npart.sum())} groups {npart.reshape(part.shape[0], -1).any(1).nonzero().flatten()[:8].tolist()}",
          flush=True)
