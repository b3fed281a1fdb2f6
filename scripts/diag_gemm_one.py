"""One GEMM shape through the NT conv kernel (1x1 conv over an [M,1,1,C] image), for PMC runs:
python scripts/diag_gemm_one.py M CIN KOUT [iters] [stats 0/1]"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd.ops import native  # noqa: E402

m, c, k = (int(v) for v in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
stats = (sys.argv[5] != "0") if len(sys.argv) > 5 else True
C = native()
dev = torch.device("cuda:0")
x = torch.randn(m, 1, 1, c, device=dev).to(torch.bfloat16)
w = (torch.randn(k, c, 1, 1, device=dev) / c ** 0.5).contiguous(memory_format=torch.channels_last)
wp = C.pack_weight(w, c)
for _ in range(3):
    C.conv_fwd(x, wp, 1, 0, stats)
torch.cuda.synchronize()
s, e = torch.cuda.Event(True), torch.cuda.Event(True)
s.record()
for _ in range(iters):
    C.conv_fwd(x, wp, 1, 0, stats)
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) / iters * 1e3
print(f"M={m} C={c} K={k} stats={stats}: {us:.1f} us, {2.0 * m * c * k / us / 1e6:.0f} TFLOP/s", flush=True)
