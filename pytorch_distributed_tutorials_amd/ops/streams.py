"""Side stream for weight-gradient GEMMs.

In a conv unit's backward the input-gradient (dgrad) and weight-gradient (wgrad)
GEMMs are independent.  Issuing wgrad on a second HIP stream lets the two fill
each other's partial waves: a 7x7 or 14x14 layer launches fewer workgroups than
the chip has CUs, and every GEMM ends in a tail where CUs drain.  The dgrad chain
stays on the caller's stream (it is the critical path of backward).

Ordering: the side stream waits for the caller's stream before each wgrad (its
inputs are ready); the inputs are ``record_stream``-ed so the caching allocator
does not hand their memory out while the side stream still reads them -- all three
in one native call, ``C.conv_wgrad_side`` (csrc/bindings.cpp); gradient
all-reduces wait for the side stream (``Reducer.set_aux_stream``); and a callback
at the end of backward joins it into the caller's stream, so the optimizer step
sees every gradient.

One join per backward pass suffices: ``begin`` queues it for the first block of a
graph task only.  (Handing a block's wgrads over in one batch instead of one per
wgrad was measured slower: 11.9k vs 12.0k img/s, the wgrads lose their overlap
with their own block's dgrad chain.)
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch

_enabled = True
_branch_enabled = True
_streams: Dict[int, torch.cuda.Stream] = {}
_branch_streams: Dict[int, torch.cuda.Stream] = {}
_joined_task = [None]  # graph task whose end-of-backward join is already queued


def set_enabled(on: bool) -> None:
    global _enabled
    _enabled = on


def wgrad_stream(device: torch.device) -> Optional[torch.cuda.Stream]:
    if not _enabled or device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _streams[idx] = s
    return s


_critical: Dict[int, torch.cuda.Stream] = {}


def critical_stream(device: torch.device) -> Optional[torch.cuda.Stream]:
    """High-priority stream for the training step's critical path (forward, the dgrad chain,
    optimizer): the side streams (weight gradients, projection branch) run at normal priority, so
    when both have workgroups waiting the dispatcher hands CUs to the critical path first and the
    side work fills what is left.  Measured on MI355X, ResNet-50 b256 (r3l, same box): 20.01 ->
    19.56 ms/step.  (Confining the weight-gradient stream to a CU mask instead -- 128 or 192 of
    256 CUs, ``C.cu_masked_stream`` -- was 28 ms/step.)"""
    if device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _critical.get(idx)
    if s is None:
        lo, hi = torch.cuda.Stream.priority_range()
        s = torch.cuda.Stream(device=idx, priority=min(lo, hi))
        _critical[idx] = s
    return s


def critical_priority_wanted(collective: bool, graph: bool, fp8: bool = False) -> bool:
    """Whether the step should run on :func:`critical_stream`: the eager fp8 step without gradient
    collectives (r7x, same call: 16.66 / 16.66 ms with the priority vs 16.96 / 16.91 without);
    nothing else (below).

    History: the priority paid in the plain
    single-GPU step (r3z, same box: 19.41 -> 18.95 ms) but costs far more than it gains as soon
    as the step adds cross-stream synchronisation with a normal-priority stream outside the
    compute chain: ResNet-50 with the gradient reducer (world-1 RCCL or xGMI) 19.5 -> 28.4 ms,
    its HIP-graph replay 20.7 -> 29.6 ms, ResNet-18/CIFAR graph replay 2.04 -> 6.34 ms; every
    small main-stream kernel is ~35 us longer in the kernel trace
    (``profiles/r3z_priority_vs_sync.md``).

    Off by default since round 5: with the BN backward folded into the input gradient and the
    forward statistics taken in the conv epilogue, the plain step is FASTER at normal priority
    (r7q, same call, two runs each: 18.11 / 18.08 ms vs 18.22 / 18.16 ms with the priority), and
    the N>1 code path at world 1 (``--force-comm``, normal priority) is within 0.2 % of either
    (RCCL 18.26 / 18.20, xGMI 18.16 / 18.15; ``profiles/r7q_priority_ab.jsonl``).  So every world
    size now runs the same stream setup.  ``PDT_MAIN_PRIO=1`` / ``=0`` forces it on / off."""
    e = os.environ.get("PDT_MAIN_PRIO", "auto")
    if e in ("0", "1"):
        return e == "1"
    return fp8 and not collective and not graph


def use_critical_stream(device: torch.device, collective: bool = False,
                        graph: bool = False, fp8: bool = False) -> Optional[torch.cuda.Stream]:
    """Make :func:`critical_stream` the current stream of ``device`` when
    :func:`critical_priority_wanted` says so (call once, before the model and its buffers are
    touched, so every later op orders on it)."""
    if not critical_priority_wanted(collective, graph, fp8):
        return None
    s = critical_stream(device)
    if s is not None:
        torch.cuda.set_stream(s)
    return s


def set_branch_enabled(on: bool) -> None:
    global _branch_enabled
    _branch_enabled = on


def branch_stream(device: torch.device) -> Optional[torch.cuda.Stream]:
    """Stream for the projection-shortcut branch of a downsampling block :
    the shortcut conv + BN statistics in forward, and its BN backward + input gradient in
    backward, run concurrently with the main chain's first units and join before the unit that
    consumes them.  They fill the CUs the main chain's GEMMs leave idle (grids of 49 x 2^k
    tiles on 256 CUs: ~77 % wave efficiency in ResNet layers 2-4)."""
    if not _branch_enabled or device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _branch_streams.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _branch_streams[idx] = s
    return s


def fork(branch: torch.cuda.Stream, *inputs: torch.Tensor) -> torch.cuda.Stream:
    """Order ``branch`` after the caller's stream and keep ``inputs`` (caller-stream tensors
    the branch reads) alive for it; returns the caller's stream."""
    main = torch.cuda.current_stream(branch.device)
    branch.wait_stream(main)
    for t in inputs:
        if t is not None:
            t.record_stream(branch)
    return main


def join(branch: torch.cuda.Stream, main: torch.cuda.Stream, *outputs: torch.Tensor) -> torch.cuda.Event:
    """Event at the branch's current end, for ``main.wait_event`` where its results are needed;
    ``outputs`` (branch-allocated tensors main reads) are kept alive for main."""
    ev = torch.cuda.Event()
    ev.record(branch)
    for t in outputs:
        if t is not None:
            t.record_stream(main)
    return ev


def begin(device: torch.device) -> Optional[torch.cuda.Stream]:
    """Called inside a backward that will put work on the side stream: queues the join of the
    side stream into the caller's stream at the end of this backward pass (once per pass: the
    graph task id tells passes apart, so an aborted pass cannot suppress the next one's join)."""
    s = wgrad_stream(device)
    if s is None:
        return None
    task = (torch._C._current_graph_task_id(), device.index)
    if task[0] < 0 or _joined_task[0] != task:
        _joined_task[0] = task
        cur = torch.cuda.current_stream(device)
        torch.autograd.Variable._execution_engine.queue_callback(lambda: cur.wait_stream(s))
    return s
