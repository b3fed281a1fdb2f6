"""Isolated timing of the folded-BN weight kernel (C.bn_fold_weights) at the ResNet-50 last-unit
shapes (C = 64..512, K = 4C), to compare with its in-step duration in a kernel trace."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd.ops.fused import native  # noqa: E402

C = native()
dev = torch.device("cuda:0")
for c in (64, 128, 256, 512):
    k = 4 * c
    wt = (torch.randn(c, k, device=dev) * 0.05).to(torch.bfloat16)
    stats = torch.stack([torch.randn(k) * 0.1, torch.rand(k) + 0.5, torch.ones(k), torch.zeros(k)]).to(dev).contiguous()
    gamma = torch.rand(k, device=dev) + 0.5
    sums = torch.randn(2, k, device=dev)
    for _ in range(5):
        C.bn_fold_weights(wt, stats, gamma, sums, 1000)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    s.record()
    for _ in range(n):
        C.bn_fold_weights(wt, stats, gamma, sums, 1000)
    e.record()
    torch.cuda.synchronize()
    print(f"C={c} K={k}: {s.elapsed_time(e) / n * 1000:.1f} us per call (coef + fold launches)")
