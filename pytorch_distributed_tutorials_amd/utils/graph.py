"""Whole-training-step capture in a HIP graph.

A ResNet training step is ~400 kernel launches (conv GEMMs, BN passes, the
reducer's bucketed all-reduces on the RCCL stream, the weight-gradient side
stream, the fused optimizer).  Issued one by one from Python they cost CPU time
that, for small per-GPU work (the reference's ResNet-18 on 32x32 CIFAR) or many
GPUs (launch jitter delays the collectives every rank waits on), shows up in the
step time.  ``CapturedStep`` records one full step -- zero_grad, forward, loss,
backward with the DDP all-reduces, optimizer -- into a graph once and then
replays it with a single launch; inputs are fed through static tensors.

Everything the step enqueues is capturable: our kernels launch on the current
stream, the RCCL and side streams join the capture through events, allocations
come from the graph's private pool.  The CPU-side bookkeeping (reducer hooks,
BN counters, weight-mirror versions) runs during capture only -- valid because
the ResNet graph is static (same shapes, same buckets, every step).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class CapturedStep:
    def __init__(self, step_fn: Callable[[], torch.Tensor], warmup: int = 3,
                 pool: Optional[tuple] = None):
        self.step_fn = step_fn
        self.warmup = warmup
        self.pool = pool
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.output: Optional[torch.Tensor] = None

    def capture(self) -> None:
        # warm up on a side stream (lazy init, allocator pools, kernel attributes), then capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self.step_fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=self.pool):
            self.output = self.step_fn()
        torch.cuda.synchronize()

    def __call__(self) -> torch.Tensor:
        if self.graph is None:
            self.capture()
        self.graph.replay()
        return self.output
