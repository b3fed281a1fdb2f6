"""Stem forward kernel timing (ResNet-50 stem at batch 256, 224 px), per PDT_STEM_DBG variant."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd.ops import native  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000.0


def main():
    C = native()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    x = torch.randn(n, 3, 224, 224, device="cuda")
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    ref = None
    for dbg in [int(v) for v in os.environ.get("STEM_VARIANTS", "0").split(",")]:
        os.environ["PDT_STEM_DBG"] = str(dbg)
        us = timeit(lambda: C.stem_conv_fwd(x, w, 2, 3, True))
        err = ""
        if dbg & 7 == 0:
            out = C.stem_conv_fwd(x, w, 2, 3, True)
            torch.cuda.synchronize()
            if ref is None:
                ref = [t.clone() for t in out[1:3]]
            else:
                err = " y_diff=%g part_diff=%g" % (float((out[1].float() - ref[0].float()).abs().max()),
                                                   float((out[2] - ref[1]).abs().max()))
        print(f"dbg={dbg} stem_conv_fwd (image relayout + conv + partials) {us:.1f} us{err}", flush=True)
    os.environ["PDT_STEM_DBG"] = "0"


if __name__ == "__main__":
    main()
