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

from typing import List, Optional, Sequence

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


def split_tail(plan: List[List[int]], sizes_bytes: Sequence[int], last_cap_bytes: int) -> List[List[int]]:
    """Cap the LAST bucket: carve the trailing items (in readiness order) whose total stays
    within ``last_cap_bytes`` into a final bucket of their own.  The item that would cross the
    cap stays in the previous bucket, so the tail bucket is <= the cap unless its single last
    item alone exceeds it (then that item is the tail).  ``plan`` holds positions."""
    if not plan or last_cap_bytes <= 0:
        return plan
    last = plan[-1]
    total = sum(int(sizes_bytes[p]) for p in last)
    if total <= last_cap_bytes or len(last) == 1:
        return plan
    tail: List[int] = []
    acc = 0
    for p in reversed(last):
        if tail and acc + int(sizes_bytes[p]) > last_cap_bytes:
            break
        tail.append(p)
        acc += int(sizes_bytes[p])
    tail.reverse()
    head = last[:len(last) - len(tail)]
    return plan[:-1] + ([head] if head else []) + [tail]


def ddp_bucket_plan(param_sizes_bytes: Sequence[int], bucket_cap_mb: float = 25.0,
                    first_bucket_mb: float = 1.0,
                    last_bucket_mb: Optional[float] = None) -> List[List[int]]:
    """Buckets of parameter INDICES (definition order) in reverse-definition order.

    ``first_bucket_mb`` caps the bucket launched first (torch: 1 MiB); ``last_bucket_mb``
    (None = torch behaviour, no cap) caps the bucket launched LAST -- the one holding the
    stem/layer1 gradients, produced at the very end of backward, whose all-reduce is the only
    one nothing can hide (see ``tail_time_us``)."""
    n = len(param_sizes_bytes)
    order = list(reversed(range(n)))
    caps = [int(first_bucket_mb * MiB), int(bucket_cap_mb * MiB)]
    sizes = [param_sizes_bytes[i] for i in order]
    plan = plan_buckets(sizes, caps)
    if last_bucket_mb is not None:
        plan = split_tail(plan, sizes, int(last_bucket_mb * MiB))
    return [[order[p] for p in b] for b in plan]


# ---------------------------------------------------------------------------------------------
# xGMI tail model
# ---------------------------------------------------------------------------------------------
XGMI_LINK_GBPS = 153.0   # one xGMI link, one direction (MI355X, 8-GPU node)
XGMI_LINKS = 7           # point-to-point links per GPU in a fully connected 8-GPU node
RCCL_LAUNCH_US = 12.0    # per-collective fixed cost (launch + ring setup), order of magnitude


def allreduce_us(nbytes: int, world: int, links_used: int = 1, latency_us: float = RCCL_LAUNCH_US,
                 link_gbps: float = XGMI_LINK_GBPS) -> float:
    """Analytic all-reduce time: a ring moves 2(n-1)/n of the buffer over each GPU's busiest
    link; RCCL's channels spread that over ``links_used`` of the 7 links (1 = a single ring,
    7 = every link busy).  Returns microseconds."""
    if world <= 1:
        return latency_us
    wire = 2.0 * (world - 1) / world * nbytes
    return latency_us + wire / (links_used * link_gbps * 1e3)


def tail_time_us(plan_bytes: Sequence[int], world: int, links_used: int = 1) -> float:
    """Exposed all-reduce time after the last gradient is produced: the last bucket's
    all-reduce cannot overlap any backward kernel (everything before it can)."""
    if not plan_bytes:
        return 0.0
    return allreduce_us(int(plan_bytes[-1]), world, links_used)


def auto_last_bucket_mb(param_sizes_bytes: Sequence[int], world: int, bucket_cap_mb: float = 25.0,
                        first_bucket_mb: float = 1.0, links_used: int = XGMI_LINKS,
                        candidates: Sequence[float] = (0.25, 0.5, 1.0, 2.0, 4.0, 8.0, 16.0)) -> Optional[float]:
    """The last-bucket cap the tail model prefers for this model and world size (None = no cap).

    The last bucket's all-reduce is the only one no backward kernel hides (``tail_time_us``), so a
    smaller last bucket shortens the step; every extra bucket costs one more collective launch,
    counted here at a quarter of ``RCCL_LAUNCH_US`` (it overlaps backward, but serialises on the
    comm stream).  World 1 has no all-reduce: None."""
    if world <= 1:
        return None
    base = ddp_bucket_plan(param_sizes_bytes, bucket_cap_mb, first_bucket_mb, None)

    def cost(cap):
        plan = ddp_bucket_plan(param_sizes_bytes, bucket_cap_mb, first_bucket_mb, cap)
        nbytes = [sum(int(param_sizes_bytes[i]) for i in b) for b in plan]
        return tail_time_us(nbytes, world, links_used) + 0.25 * RCCL_LAUNCH_US * (len(plan) - len(base))

    best, best_cost = None, cost(None)
    for cap in candidates:
        c = cost(cap)
        if c < best_cost - 1e-9:
            best, best_cost = cap, c
    return best
