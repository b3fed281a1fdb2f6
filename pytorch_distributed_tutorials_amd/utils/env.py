"""Launcher environment contract.

The reference script is meant to be started by ``torch.distributed.launch`` /
``torchrun`` and reads ``--local_rank`` from argv (``resnet/main.py:52``).  The
elastic agent exports ``RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT,
LOCAL_WORLD_SIZE, GROUP_RANK`` (torch/distributed/elastic/agent/server/
local_elastic_agent.py:306-319).  This module resolves that contract in one
place so the CLI, the launcher and bench.py agree.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional


@dataclass(frozen=True)
class DistEnv:
    rank: int
    local_rank: int
    world_size: int
    local_world_size: int
    master_addr: str
    master_port: int

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def _int_env(name: str, default: int) -> int:
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    return int(v)


def dist_env(local_rank_arg: Optional[int] = None) -> DistEnv:
    """Resolve rank/world info.

    ``local_rank_arg`` (from ``--local_rank``/``--local-rank``) wins over the
    ``LOCAL_RANK`` env var, which wins over 0 (fixes reference defect D5).
    """
    world = _int_env("WORLD_SIZE", 1)
    rank = _int_env("RANK", 0)
    if local_rank_arg is not None:
        local_rank = int(local_rank_arg)
    else:
        local_rank = _int_env("LOCAL_RANK", rank if world > 1 else 0)
    return DistEnv(
        rank=rank,
        local_rank=local_rank,
        world_size=world,
        local_world_size=_int_env("LOCAL_WORLD_SIZE", world),
        master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
        master_port=_int_env("MASTER_PORT", 29500),
    )
