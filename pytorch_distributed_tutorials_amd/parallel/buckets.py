"""Gradient bucket planning.

Reproduces the layout torch DDP converges to after its iteration-1 rebuild
(``_rebuild_buckets``, torch/nn/parallel/distributed.py:1551 with caps
``[dist._DEFAULT_FIRST_BUCKET_BYTES = 1 MiB, bucket_cap_mb = 25 MiB]``): walk
parameters in reverse definition order (= the order gradients become ready in
backward), keep adding to the current bucket, close it as soon as it reaches the
current cap (the tensor that crosses the cap stays in), then move to the next cap.
For ResNet-50 that gives 5 buckets [2,049,000, 7,875,584, 6,563,840, 6,637,568,
2,431,040] elements.  Because ResNet's graph is static the
plan is fixed from iteration 0 (no single-bucket warm-up iteration).

Bucket sizes are a tunable for xGMI: each GPU has 7 point-to-point links, an
RCCL ring uses one of them per step, so per-call latency (~tens of µs) and the
size of the LAST bucket (the stem/layer1 gradients produced at the very end of
backward, whose all-reduce cannot overlap anything) matter more than the cap.
"""
from __future__ import annotations

from typing import List, Sequence

MiB = 1 << 20


def plan_buckets(sizes_bytes: Sequence[int], caps_bytes: Sequence[int]) -> List[List[int]]:
    """Greedy bucket assignment over items given in readiness order.

    Returns lists of positions (into ``sizes_bytes``).  ``caps_bytes`` is the cap
    sequence; the last cap repeats.
    """
    if not caps_bytes:
        raise ValueError("need at least one cap")
    out: List[List[int]] = []
    cur: List[int] = []
    cur_bytes = 0
    cap_i = 0
    for pos, nbytes in enumerate(sizes_bytes):
        cur.append(pos)
        cur_bytes += int(nbytes)
        if cur_bytes >= caps_bytes[cap_i]:
            out.append(cur)
            cur, cur_bytes = [], 0
            cap_i = min(cap_i + 1, len(caps_bytes) - 1)
    if cur:
        out.append(cur)
    return out


def ddp_bucket_plan(param_sizes_bytes: Sequence[int], bucket_cap_mb: float = 25.0,
                    first_bucket_mb: float = 1.0) -> List[List[int]]:
    """Buckets of parameter INDICES (definition order) in reverse-definition order."""
    n = len(param_sizes_bytes)
    order = list(reversed(range(n)))
    caps = [int(first_bucket_mb * MiB), int(bucket_cap_mb * MiB)]
    plan = plan_buckets([param_sizes_bytes[i] for i in order], caps)
    return [[order[p] for p in b] for b in plan]
