"""Rank-sharded sampler with exactly ``torch.utils.data.DistributedSampler`` semantics.

Reference usage: ``DistributedSampler(dataset=train_set)`` with all defaults
(``resnet/main.py:97``): shuffle=True, seed=0, drop_last=False, padding by
wrap-around to a multiple of the world size, rank-strided slicing
(torch/utils/data/distributed.py:107-141).  The index stream is bit-identical to
torch's (same ``torch.randperm`` generator seeding ``seed + epoch``), which the
tests check.  Unlike the reference we make ``set_epoch`` part of the trainer
loop (reference defect D6).
"""
from __future__ import annotations

import math
from typing import Iterator, List, Optional

import torch


class DistributedSampler:
    def __init__(self, dataset_len: int, num_replicas: Optional[int] = None,
                 rank: Optional[int] = None, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        if hasattr(dataset_len, "__len__"):
            dataset_len = len(dataset_len)  # accept a dataset, like torch
        if num_replicas is None or rank is None:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
                rank = dist.get_rank() if rank is None else rank
            else:
                num_replicas = 1 if num_replicas is None else num_replicas
                rank = 0 if rank is None else rank
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in [0, {num_replicas - 1}]")
        self.n = int(dataset_len)
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        self.shuffle = shuffle
        self.seed = seed
        if self.drop_last and self.n % self.num_replicas != 0:
            self.num_samples = math.ceil((self.n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(self.n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas

    def indices(self) -> List[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad <= len(idx):
                idx += idx[:pad]
            else:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        assert len(idx) == self.total_size
        idx = idx[self.rank:self.total_size:self.num_replicas]
        assert len(idx) == self.num_samples
        return idx

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices())

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
