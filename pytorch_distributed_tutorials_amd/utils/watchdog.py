"""Failure detection: a per-rank progress watchdog and fault injection.

The reference relies on the implicit NCCL process-group timeout (10 min) and
torchrun's fail-fast (no explicit failure-detection code).  A hung
peer then leaves every other rank blocked inside an RCCL kernel.  The watchdog
here is a daemon thread fed a heartbeat each step; when a rank makes no progress
for ``timeout`` seconds it reports the rank, the phase it was in and how long it
has been stuck, aborts the native RCCL communicator (``ncclCommAbort`` unblocks
kernels waiting on a dead peer) and terminates the process with
:data:`EXIT_CODE`, so the launcher's fail-fast tears the job down instead of it
hanging until the collective timeout.

Fault injection (for tests and drills): ``PDT_FAULT="rank:step:kind[,...]"``
with kind ``crash`` (raise), ``exit`` (``os._exit(3)``) or ``hang`` (sleep
forever) makes that rank fail at that training step.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, List, Optional

EXIT_CODE = 124


class Watchdog:
    def __init__(self, timeout: float, rank: int = 0, on_timeout: Optional[Callable[[], None]] = None,
                 poll: Optional[float] = None, exit_process: bool = True):
        if timeout <= 0:
            raise ValueError("watchdog timeout must be positive")
        self.timeout = float(timeout)
        self.rank = rank
        self.on_timeout = on_timeout
        self.exit_process = exit_process
        self.poll = poll if poll is not None else min(1.0, self.timeout / 4)
        self.phase = "init"
        self.fired = False
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name=f"pdt-watchdog-{rank}", daemon=True)
        self._thread.start()

    def heartbeat(self, phase: Optional[str] = None) -> None:
        self._last = time.monotonic()
        if phase is not None:
            self.phase = phase

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(timeout=5)

    def _run(self) -> None:
        while not self._stop.wait(self.poll):
            idle = time.monotonic() - self._last
            if idle > self.timeout:
                self.fired = True
                sys.stderr.write(
                    f"[watchdog] rank {self.rank}: no progress for {idle:.1f}s (limit {self.timeout:.1f}s) "
                    f"in phase '{self.phase}'; a peer rank has likely failed or hung. Aborting.\n")
                sys.stderr.flush()
                if self.on_timeout is not None:
                    try:
                        self.on_timeout()
                    except Exception as e:  # noqa: BLE001 - best effort during teardown
                        sys.stderr.write(f"[watchdog] abort hook failed: {e}\n")
                if self.exit_process:
                    os._exit(EXIT_CODE)
                return


def parse_faults(spec: Optional[str]) -> List[tuple]:
    out = []
    if not spec:
        return out
    for item in spec.split(","):
        item = item.strip()
        if not item:
            continue
        r, s, kind = item.split(":")
        if kind not in ("crash", "exit", "hang"):
            raise ValueError(f"unknown fault kind {kind!r}")
        out.append((int(r), int(s), kind))
    return out


class FaultInjector:
    def __init__(self, rank: int, spec: Optional[str] = None):
        self.rank = rank
        self.faults = [(s, k) for r, s, k in parse_faults(spec if spec is not None
                                                          else os.environ.get("PDT_FAULT"))
                       if r == rank]

    def __call__(self, step: int) -> None:
        for s, kind in self.faults:
            if s == step:
                sys.stderr.write(f"[fault] rank {self.rank}: injecting '{kind}' at step {step}\n")
                sys.stderr.flush()
                if kind == "crash":
                    raise RuntimeError(f"injected fault on rank {self.rank} at step {step}")
                if kind == "exit":
                    os._exit(3)
                while True:  # hang
                    time.sleep(3600)
