#!/usr/bin/env python3
"""Busy/idle analysis of a rocprofv3 kernel trace: per step, GPU busy time (union of kernel
intervals over all streams), per-stream busy time, and the largest idle gaps.

    python scripts/trace_gaps.py gpurun_out/prof_x/run_kernel_trace.csv [--steps 5]
"""
import argparse
import csv
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, n in iv:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            tot += cur_e - cur_s
            gaps.append((s - cur_e, cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot, gaps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--step-marker", default="stem_image_kernel",
                    help="kernel that starts a training step; the last complete step of typical length "
                         "(the bench's diagnostic steps that follow are skipped) is analysed")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.step_marker and a.step_marker in r["Kernel_Name"]]
    if len(idx) >= 2:
        spans = [(int(rows[j]["Start_Timestamp"]) - int(rows[i]["Start_Timestamp"]), i, j)
                 for i, j in zip(idx, idx[1:])]
        med = sorted(sp for sp, _, _ in spans)[len(spans) // 2]
        i0, i1 = [(i, j) for sp, i, j in spans if sp < 1.5 * med][-1]
        rows = rows[i0:i1]
        print(f"last typical step only ({len(rows)} kernels, marker {a.step_marker})")
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:90]) for r in rows]
    by_q = defaultdict(list)
    for r, x in zip(rows, iv):
        by_q[r["Queue_Id"]].append(x)
    t0 = min(s for s, _, _ in iv)
    t1 = max(e for _, e, _ in iv)
    busy, gaps = union(iv)
    print(f"span {(t1 - t0) / 1e6:.2f} ms, busy(union) {busy / 1e6:.2f} ms, idle {(t1 - t0 - busy) / 1e6:.2f} ms")
    for q, v in sorted(by_q.items()):
        b, _ = union(v)
        print(f"  queue {q}: {len(v)} kernels, busy {b / 1e6:.2f} ms")
    gaps.sort(reverse=True)
    print("largest idle gaps (us, before kernel):")
    for g, at, n in gaps[:a.top]:
        print(f"  {g / 1e3:8.1f} us at +{(at - t0) / 1e6:8.2f} ms before {n}")
    small = sum(g for g, _, _ in gaps if g < 50_000)
    print(f"sum of gaps < 50us: {small / 1e6:.2f} ms over {sum(1 for g in gaps if g[0] < 50_000)} gaps")


if __name__ == "__main__":
    main()
