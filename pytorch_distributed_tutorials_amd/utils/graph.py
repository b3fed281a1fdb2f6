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

import gc
from typing import Callable, List, Optional, Tuple

import torch


class CapturedStep:
    """Capture ``step_fn`` once (after ``warmup`` eager calls on a side stream) and replay it.

    ``period`` > 1 captures that many consecutive steps as separate graphs (sharing one memory
    pool) and replays them round-robin.  That keeps host-side state that cycles with the step
    count valid under replay: fp8 delayed scaling rotates a 3-slot amax/scale ring per step
    (``ops.fused._Q8State``), so graph k bakes in the slot indices of a step t = t0 + k.

    ``ring = (get, set)`` exposes that host state (a tuple of step counters).  Capture executes
    nothing on the device, so after capturing, the counters are put back to their pre-capture
    values and every replay advances them by one step's worth -- the host always describes what
    the device has run, and eager work between replays (an evaluation, a partial batch) uses
    the right slots.  ``in_phase()`` tells whether the next replay's baked-in slots still match
    the counters (eager work that advanced a ring by other than a multiple of its cycle breaks
    them: capture again).

    Output validity: the graphs share one private memory pool, so graph k+1 may place its
    output where graph k keeps temporaries; replaying graph k would then overwrite it.  Each
    graph therefore copies its output (the step's loss) into a static buffer allocated OUTSIDE
    the pool before capture, and ``__call__`` returns that buffer: the value of replay k stays
    valid until graph k is replayed again (``period`` calls later) -- copy it if you need it
    longer (e.g. to accumulate losses on the device over an epoch).
    """

    def __init__(self, step_fn: Callable[[], torch.Tensor], warmup: int = 3,
                 pool: Optional[tuple] = None, period: int = 1,
                 ring: Optional[Tuple[Callable[[], Tuple[int, ...]], Callable[[Tuple[int, ...]], None]]] = None,
                 cycle: int = 3):
        if period < 1:
            raise ValueError("period must be >= 1")
        self.step_fn = step_fn
        self.warmup = warmup
        self.pool = pool
        self.period = period
        self.ring = ring
        self.cycle = cycle
        self.phase_sig: List[Tuple[int, ...]] = []  # counters (mod cycle) graph k was captured at
        self.delta: Tuple[int, ...] = ()            # counter advance of one step
        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.outputs: List[torch.Tensor] = []  # static per-graph output buffers (outside the pool)
        self.calls = 0

    @property
    def graph(self) -> Optional[torch.cuda.CUDAGraph]:
        return self.graphs[0] if self.graphs else None

    def _mod(self, t: Tuple[int, ...]) -> Tuple[int, ...]:
        return tuple(v % self.cycle for v in t)

    def capture(self) -> None:
        # warm up on a side stream (lazy init, allocator pools, kernel attributes), then capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        probe = None
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                probe = self.step_fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # side-stream work the warm-up left pending (weight-layout packs) is done now; the capture
        # must not wait on its events (recorded outside the capture)
        from ..parallel.flat import forget_completed_side_packs
        forget_completed_side_packs()
        # output buffers: allocated here, before any capture, so they live outside the pool
        if probe is not None:
            self.outputs = [torch.empty_like(probe) for _ in range(self.period)]
        else:  # no eager warm-up: the step returns its loss, an fp32 scalar
            self.outputs = [torch.empty((), dtype=torch.float32, device=torch.cuda.current_device()) for _ in range(self.period)]
        # no cyclic garbage collection while capturing: a collected cycle that owns a HIP event or
        # graph (autograd contexts of earlier steps) would be destroyed inside the capture, which
        # aborts the process; collect before (and before the ring snapshot, whose entries belong to
        # live objects), and let anything created during capture wait
        gc.collect()
        start = self.ring[0]() if self.ring is not None else ()
        gc_was_on = gc.isenabled()
        gc.disable()
        try:
            self._capture_graphs()
        finally:
            if gc_was_on:
                gc.enable()
        if self.ring is not None:
            end = self.ring[0]()
            if len(end) != len(start):
                raise RuntimeError("CapturedStep: the captured step created new ring state; warm it up first")
            self.delta = tuple((e - b) // self.period for b, e in zip(start, end))
            self.ring[1](start)  # the device has run none of the captured steps yet
        torch.cuda.synchronize()

    def _capture_graphs(self) -> None:
        pool = self.pool
        for k in range(self.period):
            if self.ring is not None:
                self.phase_sig.append(self._mod(self.ring[0]()))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                out = self.step_fn()
                if out.shape != self.outputs[k].shape or out.dtype != self.outputs[k].dtype:
                    raise RuntimeError(f"CapturedStep: step output {tuple(out.shape)} {out.dtype} does not "
                                       f"match the static buffer {tuple(self.outputs[k].shape)} "
                                       f"{self.outputs[k].dtype}")
                self.outputs[k].copy_(out)
            if pool is None:
                pool = g.pool()  # later phases reuse the first graph's private pool
            self.graphs.append(g)

    def in_phase(self) -> bool:
        """False when eager work moved the host counters off the next replay's baked-in phase."""
        if not self.graphs or self.ring is None:
            return True
        cur = self.ring[0]()
        return len(cur) == len(self.delta) and self._mod(cur) == self.phase_sig[self.calls % self.period]

    def __call__(self) -> torch.Tensor:
        """Replay the next graph; returns its static output buffer (valid until that same graph
        is replayed again, ``period`` calls later)."""
        if not self.graphs:
            self.capture()
        k = self.calls % self.period
        self.calls += 1
        self.graphs[k].replay()
        if self.ring is not None:
            self.ring[1](tuple(t + d for t, d in zip(self.ring[0](), self.delta)))
        return self.outputs[k]
