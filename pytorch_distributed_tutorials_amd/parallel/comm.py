"""Process-group bootstrap and the native RCCL communicator.

``init_distributed`` is the reference's ``init_process_group(backend="nccl")``
(``resnet/main.py:74``, env:// rendezvous through TCPStore) with its defects
fixed: the device is bound with ``torch.cuda.set_device(local_rank)`` before
any collective (D9), the backend falls back to gloo on CPU, and the timeout is
configurable.  On ROCm the ``nccl`` backend is RCCL.

``native_comm`` builds the framework's own RCCL communicator (C++,
``csrc/comm/rccl_comm.cpp``) for the data-parallel hot path.  Bring-up is a two-phase
protocol over the rendezvous store, so that no rank ever enters the RCCL init alone:

1. **agree** (:func:`agree_native`): every rank publishes whether it can build the
   communicator (extension importable, device usable; rank 0 also draws the RCCL unique id and
   publishes it), then waits -- with a deadline -- for every other rank's answer.  A rank that
   never answers makes the others raise a clear "peer never reached setup" error after the
   timeout; a rank that answers "cannot" makes EVERY rank take the same decision (fall back to
   ``torch.distributed`` collectives, or raise with ``comm='rccl'``).
2. **init**: only when all ranks said yes, each one initialises its communicator with a
   deadline (``RcclComm(init_timeout=...)``; the init runs on a helper thread): a peer that
   dies between the two phases turns into an init-timeout error instead of a hang.

After init a monitor thread in the communicator watches RCCL's async error state and the
completion of every collective (``op_timeout``, ProcessGroupNCCL's 10-minute default), aborts the
communicator on failure and, with ``exit_on_error`` (the default when world > 1), ends the process
so the launcher's fail-fast tears the job down.
"""
from __future__ import annotations

import datetime
import itertools
import os
import time
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist

from ..utils.env import DistEnv, dist_env

_COMM_CACHE = {}
_UID_COUNTER = itertools.count()

# ProcessGroupNCCL's default collective timeout (torch/distributed/constants.py:21)
DEFAULT_TIMEOUT_S = 600.0


def init_distributed(backend: Optional[str] = None, local_rank: Optional[int] = None,
                     timeout_s: Optional[float] = None) -> DistEnv:
    env = dist_env(local_rank)
    use_cuda = torch.cuda.is_available() and backend != "gloo"
    if use_cuda:
        torch.cuda.set_device(env.local_rank)
    if env.world_size > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if use_cuda else "gloo"
        kw = {}
        if timeout_s is not None:
            kw["timeout"] = datetime.timedelta(seconds=timeout_s)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        dist.init_process_group(backend=backend, init_method="env://", rank=env.rank,
                                world_size=env.world_size, **kw)
    global _PG_TIMEOUT_S
    _PG_TIMEOUT_S = timeout_s
    return env


_PG_TIMEOUT_S: Optional[float] = None


def world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def backend_name(pg=None) -> str:
    if not (dist.is_available() and dist.is_initialized()):
        return "none"
    return str(dist.get_backend(pg)).lower()


@dataclass
class CommOptions:
    """Failure handling and RCCL knobs of the native communicator.

    ``init_timeout`` bounds both the cross-rank agreement and the RCCL init;
    ``op_timeout`` bounds each collective (0 = off).  ``exit_on_error`` ends the process when the
    monitor aborts the communicator (default: on when world > 1).  ``min_channels`` /
    ``max_channels`` bound the RCCL channels (rings) a collective spreads over (``ncclConfig_t``
    minCTAs / maxCTAs; 0 = RCCL's choice); the env knob ``PDT_RCCL_CHANNELS=min[,max]`` sets them
    too.  ``xgmi_blocks`` is the same budget for the direct xGMI backend: its reduce-scatter /
    all-gather kernels use at most that many workgroups beside the backward pass.
    ``wgrad_cu_reserve``: CUs the weight-gradient split-K plan leaves free for those collective
    kernels while the step all-reduces across ranks (-1 = auto: the xGMI block budget, or the RCCL
    channel cap, 16 when RCCL chooses; env ``PDT_WGRAD_RESERVE_CUS``; ``DistributedDataParallel``
    applies it)."""
    init_timeout: float = DEFAULT_TIMEOUT_S
    op_timeout: float = DEFAULT_TIMEOUT_S
    exit_on_error: Optional[bool] = None
    min_channels: int = 0
    max_channels: int = 0
    xgmi_blocks: int = 16  # CU budget of the xGMI backend's data kernels (PDT_XGMI_BLOCKS)
    wgrad_cu_reserve: int = -1

    @classmethod
    def from_env(cls, timeout: Optional[float] = None, **kw) -> "CommOptions":
        o = cls(**kw)
        t = timeout if timeout is not None else _PG_TIMEOUT_S
        if t is not None:
            o.init_timeout = o.op_timeout = float(t)
        if os.environ.get("PDT_COMM_TIMEOUT"):
            o.init_timeout = o.op_timeout = float(os.environ["PDT_COMM_TIMEOUT"])
        if os.environ.get("PDT_XGMI_BLOCKS"):
            o.xgmi_blocks = max(1, int(os.environ["PDT_XGMI_BLOCKS"]))
        if os.environ.get("PDT_WGRAD_RESERVE_CUS"):
            o.wgrad_cu_reserve = max(0, int(os.environ["PDT_WGRAD_RESERVE_CUS"]))
        ch = os.environ.get("PDT_RCCL_CHANNELS")
        if ch and not (o.min_channels or o.max_channels):
            parts = [int(x) for x in ch.split(",")]
            o.min_channels = parts[0]
            o.max_channels = parts[1] if len(parts) > 1 else parts[0]
        return o


class CommSetupError(RuntimeError):
    """Some rank cannot build the native communicator: a decision every rank reaches alike."""


class CommSetupTimeout(RuntimeError):
    """A peer never reached the native communicator bring-up (crashed / hung): not recoverable."""


@dataclass
class Agreement:
    ok: bool                      # every rank can build the communicator
    uid: Optional[bytes] = None   # RCCL unique id (when ok)
    refusals: List[str] = field(default_factory=list)  # "rank r: reason" of the ranks that cannot


def _fault_native(rank_: int) -> Optional[str]:
    """Fault injection for tests: ``PDT_FAULT_NATIVE="r[,r2]:cannot|never"`` makes those ranks
    report that they cannot build the communicator, or never reach the agreement (sleep)."""
    spec = os.environ.get("PDT_FAULT_NATIVE")
    if not spec:
        return None
    ranks, _, kind = spec.partition(":")
    if str(rank_) in ranks.split(","):
        return kind or "cannot"
    return None


def agree_native(store, rank_: int, world: int, can_build: bool, reason: str = "",
                 timeout: float = DEFAULT_TIMEOUT_S, tag: Optional[str] = None,
                 draw_uid=None) -> Agreement:
    """Cross-rank agreement on building the native communicator (phase 1, see module doc).

    Every rank sets ``<tag>/ok/<rank>`` to "1" or "0:<reason>"; rank 0 also sets ``<tag>/uid``
    (drawn by ``draw_uid()`` when it can build).  Then every rank waits for all ``ok`` keys with
    ``timeout``; a missing rank raises :class:`CommSetupTimeout` naming it."""
    tag = tag or f"pdt/rccl/{next(_UID_COUNTER)}"
    fault = _fault_native(rank_)
    if fault == "never":
        time.sleep(10 * timeout + 60)  # a rank that never reaches setup (killed by the test)
    if fault == "cannot":
        can_build, reason = False, "fault injection (PDT_FAULT_NATIVE)"
    if rank_ == 0:
        uid = b""
        if can_build and draw_uid is not None:
            try:
                uid = draw_uid()
            except Exception as e:  # noqa: BLE001 -- reported to every rank below
                can_build, reason = False, f"ncclGetUniqueId failed: {e}"
        store.set(f"{tag}/uid", uid)
    store.set(f"{tag}/ok/{rank_}", "1" if can_build else f"0:{reason}")
    keys = [f"{tag}/ok/{r}" for r in range(world)]
    t0 = time.monotonic()
    missing = list(range(world))
    # poll key by key (store.check is non-blocking) so a timeout can name the missing ranks
    while missing:
        missing = [r for r in missing if not store.check([keys[r]])]
        if not missing:
            break
        if time.monotonic() - t0 > timeout:
            raise CommSetupTimeout(
                f"rank {rank_}: ranks {missing} never reached the RCCL communicator setup within "
                f"{timeout:.1f}s (crashed, hung, or took another code path); giving up instead of "
                "entering the RCCL init alone")
        time.sleep(0.01)
    refusals = []
    for r in range(world):
        v = store.get(keys[r]).decode()
        if v != "1":
            refusals.append(f"rank {r}: {v[2:] if v.startswith('0:') else v}")
    if refusals:
        return Agreement(False, None, refusals)
    return Agreement(True, store.get(f"{tag}/uid"), [])


def _can_build(device: torch.device) -> tuple:
    from ..ops._ext import native_available
    if device.type != "cuda":
        return False, "not a GPU device"
    if not native_available():
        return False, "native extension not importable"
    return True, ""


def native_comm(device: torch.device, pg=None, options: Optional[CommOptions] = None,
                agreement: Optional[Agreement] = None):
    """The RCCL communicator of this process for ``pg`` (cached).

    Without an initialised process group (a single-process run) this is a world-1 RCCL
    communicator whose unique id never leaves the process: every collective of the
    data-parallel path still runs through RCCL (the forced-reducer mode of
    ``DistributedDataParallel``, used to execute and test that path on one GPU).

    With a process group, runs the agreement (unless ``agreement`` is given) and raises
    :class:`CommSetupError` on every rank when any rank cannot build the communicator."""
    from ..ops._ext import native
    key = (id(pg), device.index)
    if key in _COMM_CACHE:
        return _COMM_CACHE[key]
    o = options or CommOptions.from_env()
    if not (dist.is_available() and dist.is_initialized()):
        if pg is not None:
            raise RuntimeError("native_comm: a process group was given but none is initialised")
        C = native()
        comm = C.RcclComm(C.RcclComm.unique_id(), 0, 1, device.index, init_timeout=o.init_timeout,
                          op_timeout=o.op_timeout, exit_on_error=bool(o.exit_on_error),
                          min_channels=o.min_channels, max_channels=o.max_channels)
        _COMM_CACHE[key] = comm
        return comm
    ws = dist.get_world_size(pg)
    rk = dist.get_rank(pg)
    if agreement is None:
        ok, why = _can_build(device)
        agreement = agree_native(dist.distributed_c10d._get_default_store(), rk, ws, ok, why,
                                 timeout=o.init_timeout, draw_uid=lambda: native().RcclComm.unique_id())
    if not agreement.ok:
        raise CommSetupError("native RCCL communicator not built on any rank: " + "; ".join(agreement.refusals))
    C = native()
    exit_on_error = ws > 1 if o.exit_on_error is None else o.exit_on_error
    comm = C.RcclComm(agreement.uid, rk, ws, device.index, init_timeout=o.init_timeout,
                      op_timeout=o.op_timeout, exit_on_error=exit_on_error,
                      min_channels=o.min_channels, max_channels=o.max_channels)
    _COMM_CACHE[key] = comm
    return comm


def destroy() -> None:
    _COMM_CACHE.clear()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def wgrad_cu_reserve(opts: CommOptions, xgmi: bool, collective_world: int) -> int:
    """CUs to keep out of the weight-gradient split-K plan (csrc/kernels/wgrad.hip wg_cus): none
    unless gradients are all-reduced across ranks (or a world-1 run rehearses a larger world)."""
    if opts.wgrad_cu_reserve >= 0:
        return opts.wgrad_cu_reserve
    if collective_world <= 1:
        return 0
    if xgmi:
        return opts.xgmi_blocks
    return opts.max_channels if opts.max_channels > 0 else 16
