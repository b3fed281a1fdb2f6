#!/usr/bin/env python3
"""Does an RCCL call on our communicator block the host?

Queues a long chain of GPU work on the current stream, then issues collectives on the comm
stream (the reducer's pattern: comm waits for the current stream, then all-reduce) and reports
the HOST time per call.  A call that takes about as long as the queued GPU work means the
host thread waited for the device -- which serialises the data-parallel step.

    python scripts/diag_comm.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_tutorials_amd.parallel import comm as pcomm  # noqa: E402


def busy(dev, ms_target=40.0):
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        a = a @ a * 1e-3
    torch.cuda.synchronize()
    per = (time.perf_counter() - t) / 10 * 1e3
    n = max(1, int(ms_target / per))
    return a, n, per


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    c = pcomm.native_comm(dev)
    x = torch.randn(8 << 20, device=dev)
    a, n, per = busy(dev)
    print(f"matmul {per:.2f} ms, queue {n} -> ~{n * per:.0f} ms of GPU work")
    for label, op, wait in [("avg+wait", "avg", True), ("sum+wait", "sum", True), ("avg nowait", "avg", False),
                            ("sum nowait", "sum", False)]:
        for _ in range(n):
            a = a @ a * 1e-3
        t0 = time.perf_counter()
        times = []
        for _ in range(5):
            t = time.perf_counter()
            c.all_reduce(x, op, wait)
            times.append((time.perf_counter() - t) * 1e3)
        t1 = time.perf_counter()
        c.current_wait_comm()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{label:11s}: host per call {['%.3f' % v for v in times]} ms, issue {1e3 * (t1 - t0):.2f} ms, "
              f"drain {1e3 * (t2 - t1):.2f} ms")
    # event record / stream wait alone
    for _ in range(n):
        a = a @ a * 1e-3
    t = time.perf_counter()
    for _ in range(5):
        c.comm_wait_current()
    print(f"comm_wait_current x5: {1e3 * (time.perf_counter() - t):.3f} ms")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
