"""Headroom check: our NT conv kernel on 1x1/s1 convs (a plain GEMM in NHWC) vs hipBLASLt
(torch.matmul, bf16) on the same GEMM shapes.  Prints per-shape us and TFLOP/s for both."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd.ops import native  # noqa: E402

C = native()
dev = torch.device("cuda:0")
SHAPES = [  # (M, C_in, K_out)
    (802816, 64, 256), (802816, 256, 64), (200704, 128, 512), (200704, 512, 128),
    (50176, 256, 1024), (50176, 1024, 256), (12544, 512, 2048), (12544, 2048, 512),
    (200704, 1152, 128), (50176, 2304, 256), (12544, 4608, 512), (4096, 4096, 4096),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


if len(sys.argv) > 3:  # one shape: M CIN KOUT
    SHAPES = [tuple(int(v) for v in sys.argv[1:4])]
print("M,Cin,Kout,ours_us,ours_TF,blas_us,blas_TF")
for (m, c, k) in SHAPES:
    x = torch.randn(m, c, device=dev).to(torch.bfloat16)
    w = (torch.randn(k, c, device=dev) / c ** 0.5).to(torch.bfloat16)
    fl = 2.0 * m * c * k
    # ours: 1x1 conv over an [m, 1, 1, c] NHWC image, forward with BN statistics epilogue
    x4 = x.view(m, 1, 1, c)
    w4 = w.float().view(k, c, 1, 1).contiguous(memory_format=torch.channels_last)
    wp = C.pack_weight(w4, c)
    t_ours = timeit(lambda: C.conv_fwd(x4, wp, 1, 0, True))
    t_blas = timeit(lambda: torch.matmul(x, w.t()))
    print(f"{m},{c},{k},{t_ours:.1f},{fl / t_ours / 1e6:.0f},{t_blas:.1f},{fl / t_blas / 1e6:.0f}", flush=True)
