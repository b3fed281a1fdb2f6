"""Step metrics: device step time, throughput, all-reduce time and its exposed tail.

The reference only prints per-epoch banners (``resnet/main.py:107,113-115``).
The trainer adds per-step throughput plus the two numbers that matter for DDP
scaling over xGMI: how long the bucketed all-reduces took, and how much of that
was *exposed* (the comm tail that outlasted backward compute, i.e. what the
overlap failed to hide).  Comm figures come from HIP events the native reducer
records on the RCCL stream (``Reducer.set_timing``); they are absent on gloo.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import List, Optional

import torch


@dataclass
class StepStats:
    step_ms: List[float] = field(default_factory=list)
    comm_ms: List[float] = field(default_factory=list)
    exposed_ms: List[float] = field(default_factory=list)

    def summary(self, images_per_step: int) -> dict:
        def mean(v):
            return sum(v) / len(v) if v else None
        ms = mean(self.step_ms)
        return {
            "steps": len(self.step_ms),
            "step_ms": ms,
            "img_per_s": (images_per_step * 1000.0 / ms) if ms else None,
            "comm_ms": mean(self.comm_ms),
            "exposed_comm_ms": mean(self.exposed_ms),
        }


class StepTimer:
    """Wall-clock step timer that synchronizes only at report time.

    ``tick()`` after each step records host time; ``report()`` synchronizes the
    device once and attributes the elapsed time evenly over the steps since the
    last report (exact for a steady loop, and it never serializes the loop).
    """

    def __init__(self, device: torch.device, ddp=None):
        self.device = device
        self.ddp = ddp
        self.stats = StepStats()
        self._t0 = None
        self._n = 0

    def start(self) -> None:
        self._sync()
        self._t0 = time.perf_counter()
        self._n = 0

    def tick(self) -> None:
        self._n += 1

    def _sync(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def report(self) -> Optional[dict]:
        if self._t0 is None or self._n == 0:
            return None
        self._sync()
        t = time.perf_counter()
        per = (t - self._t0) * 1000.0 / self._n
        self.stats.step_ms.extend([per] * self._n)
        comm = self.ddp.comm_stats() if self.ddp is not None else None
        if comm is not None:
            self.stats.comm_ms.append(comm["comm_ms"])
            self.stats.exposed_ms.append(comm["exposed_ms"])
        self._t0, self._n = t, 0
        out = {"step_ms": per}
        if comm is not None:
            out.update(comm)
        return out
