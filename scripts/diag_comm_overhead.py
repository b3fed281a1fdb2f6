"""Does a live RCCL communicator slow the compute stream's small kernels?

The world-1 forced-reducer step (bench.py --force-comm) measured ~28 ms vs ~19 ms, with every
small main-stream kernel ~35 us longer in the kernel trace.  This times a chain of tiny kernels
(torch adds on a 4 KB tensor) before and after each piece of the forced path is set up:
creating the communicator, running one collective, and recording an event per kernel.

usage: python scripts/diag_comm_overhead.py [--n 2000]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd.ops import _ext


def chain(x, n, ev=None):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        x.add_(1.0)
        if ev is not None:
            ev.record()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6 / n


def cross(n, prio_main, back, every=10):
    """Tiny kernels on a `main` stream (high priority if prio_main); every `every` kernels the
    normal-priority `other` stream waits for main and runs one kernel, and (back) main waits for
    other again -- the reducer's comm_wait_current / current_wait_comm pattern."""
    lo, hi = torch.cuda.Stream.priority_range()
    main = torch.cuda.Stream(priority=min(lo, hi) if prio_main else 0)
    other = torch.cuda.Stream()
    x = torch.zeros(1024, device="cuda")
    y = torch.zeros(1024, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        with torch.cuda.stream(main):
            x.add_(1.0)
        if i % every == every - 1:
            other.wait_stream(main)
            with torch.cuda.stream(other):
                y.add_(1.0)
            if back:
                main.wait_stream(other)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6 / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    a = ap.parse_args()
    C = _ext.native()
    x = torch.zeros(1024, device="cuda")
    ev = torch.cuda.Event()
    out = {}
    chain(x, 200)
    out["base_us"] = chain(x, a.n)
    out["base_event_us"] = chain(x, a.n, ev)
    comm = C.RcclComm(C.RcclComm.unique_id(), 0, 1, 0, init_timeout=60.0)
    out["comm_us"] = chain(x, a.n)
    y = torch.ones(1 << 20, device="cuda")
    comm.all_reduce(y, "sum")
    comm.synchronize()
    out["after_coll_us"] = chain(x, a.n)
    out["after_coll_event_us"] = chain(x, a.n, ev)
    time.sleep(0.2)  # the monitor thread polls every 50 ms
    out["after_sleep_us"] = chain(x, a.n)
    del comm
    out["after_destroy_us"] = chain(x, a.n)
    for prio in (False, True):
        for back in (False, True):
            out[f"cross_prio{int(prio)}_back{int(back)}_us"] = cross(a.n, prio, back)
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()
