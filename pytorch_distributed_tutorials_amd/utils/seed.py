"""Seeding / determinism (reference ``set_random_seeds``, ``resnet/main.py:16-21``).

Same seed on every rank for torch, numpy and ``random``.  The reference flips
``cudnn.deterministic``/``benchmark``; on ROCm those steer MIOpen, which the
native path does not use, so we also record a framework-level flag that makes
the native kernels pick deterministic (non-atomic) reductions.
"""
from __future__ import annotations

import random

import numpy as np
import torch

_DETERMINISTIC = False  # until set_random_seeds() asks for it (the reference does)


def set_random_seeds(seed: int = 0, deterministic: bool = True) -> None:
    global _DETERMINISTIC
    torch.manual_seed(seed)
    torch.backends.cudnn.deterministic = deterministic
    torch.backends.cudnn.benchmark = not deterministic
    np.random.seed(seed)
    random.seed(seed)
    _DETERMINISTIC = deterministic


def deterministic() -> bool:
    return _DETERMINISTIC
