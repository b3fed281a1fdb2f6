"""Direct xGMI gradient all-reduce backend (``DistributedDataParallel(comm="xgmi")``).

The reference reduces gradients through ProcessGroupNCCL (``resnet/main.py:80``), i.e. RCCL's
ring/tree algorithms.  On an 8x MI355X node every GPU has 7 point-to-point xGMI links, and a
ring moves each byte over one link per step.  This backend instead maps every
rank's flat gradient buffer into every other rank (IPC handles exchanged through the rendezvous
store) and all-reduces a bucket as a one-hop reduce-scatter (each rank sums its 1/W shard by
reading all W-1 peers at once) followed by a one-hop all-gather -- all links busy in both phases.
Kernels: ``csrc/kernels/xgmi.hip``; communicator: ``csrc/comm/xgmi_comm.cpp``.

Bring-up follows the same rules as the RCCL communicator (``parallel/comm.py``): every rank
publishes its handles (or a refusal) to the store, waits for all peers with a deadline, and only
then maps them; waits inside the all-reduce kernels are bounded too (an error code, never a hung
GPU), and the reducer raises that error at the next bucket.
"""
from __future__ import annotations

import itertools
import time
import torch
import torch.distributed as dist

from .comm import CommSetupError, CommSetupTimeout, DEFAULT_TIMEOUT_S

_TAG = itertools.count()


def xgmi_comm(device: torch.device, numel: int, nbuckets: int, pg=None,
              timeout: float = DEFAULT_TIMEOUT_S, wire: str = "fp32", max_blocks: int = 16,
              exit_on_error=None):
    """Create this rank's ``XgmiComm`` and map every peer's buffers (collective over ``pg``).

    ``wire``: "fp32" or "bf16" (half the xGMI bytes; fp32 sums); ``max_blocks``: CU budget of
    the data kernels; ``exit_on_error`` (default: world > 1): the host monitor ends the process
    when a bounded wait fails or a peer signals that it failed."""
    from ..ops._ext import native
    C = native()
    if not (dist.is_available() and dist.is_initialized()):
        comm = C.XgmiComm(0, 1, device.index, numel, nbuckets, timeout, wire, max_blocks,
                          bool(exit_on_error))
        comm.link_local([comm])
        return comm
    rank, world = dist.get_rank(pg), dist.get_world_size(pg)
    if exit_on_error is None:
        exit_on_error = world > 1
    store = dist.distributed_c10d._get_default_store()
    tag = f"pdt/xgmi/{next(_TAG)}"
    comm, err = None, ""
    try:
        comm = C.XgmiComm(rank, world, device.index, numel, nbuckets, timeout, wire, max_blocks,
                          bool(exit_on_error))
        store.set(f"{tag}/h/{rank}", b"1" + comm.ipc_handles())
    except Exception as e:  # noqa: BLE001 -- reported to every rank
        err = f"{type(e).__name__}: {e}"
        store.set(f"{tag}/h/{rank}", b"0" + err.encode())
    keys = [f"{tag}/h/{q}" for q in range(world)]
    t0 = time.monotonic()
    missing = list(range(world))
    while missing:
        missing = [q for q in missing if not store.check([keys[q]])]
        if missing and time.monotonic() - t0 > timeout:
            raise CommSetupTimeout(f"rank {rank}: ranks {missing} never published their xGMI buffers within "
                                   f"{timeout:.1f}s")
        if missing:
            time.sleep(0.01)
    vals = [store.get(k) for k in keys]
    bad = [f"rank {q}: {v[1:].decode(errors='replace')}" for q, v in enumerate(vals) if v[:1] != b"1"]
    if bad:
        raise CommSetupError("xGMI communicator not built on every rank: " + "; ".join(bad))
    comm.open_peers([v[1:] for v in vals])
    # nobody may signal a peer before that peer has mapped everything: one more store round
    store.set(f"{tag}/mapped/{rank}", b"1")
    t0 = time.monotonic()
    while not all(store.check([f"{tag}/mapped/{q}"]) for q in range(world)):
        if time.monotonic() - t0 > timeout:
            raise CommSetupTimeout(f"rank {rank}: a peer never finished mapping the xGMI buffers")
        time.sleep(0.01)
    return comm


def local_group(device: torch.device, numel: int, nbuckets: int, world: int, timeout: float = 10.0,
                wire: str = "fp32", max_blocks: int = 16):
    """``world`` in-process ranks linked by raw pointers (no IPC): tests of the kernels and the
    protocol on one GPU without separate processes."""
    from ..ops._ext import native
    C = native()
    comms = [C.XgmiComm(q, world, device.index, numel, nbuckets, timeout, wire, max_blocks, False)
             for q in range(world)]
    for c in comms:
        c.link_local(comms)
    return comms


def reduce_local_group(comms, bucket: int, offset: int, count: int, average: bool = True) -> None:
    """Enqueue one bucket on every in-process rank (each on its own comm stream), phase-major:
    streams of one process may share a hardware queue, so a rank's bounded wait must never be
    queued ahead of the signal of the rank it waits for."""
    for ph in range(6):
        for c in comms:
            c.reduce_bucket_phases(bucket, offset, count, average, ph, ph)
