#!/usr/bin/env python3
"""Every kernel of the last complete training step in a rocprofv3 kernel trace, in issue order,
with stream, grid and duration (scripts/trace_breakdown.py aggregates; this lists).

    python scripts/step_kernels.py run_kernel_trace.csv [--marker sgd_kernel] [--stream N] [--top K]
"""
import argparse
import csv
import re


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "").replace("pdt::", "")
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--stream", type=int, default=None)
    ap.add_argument("--top", type=int, default=0, help="only the K longest kernels")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(ends) < 2:
        raise SystemExit("need two step markers")
    step = rows[ends[-2] + 1: ends[-1] + 1]
    t0 = int(step[0]["Start_Timestamp"])
    out = []
    for r in step:
        s = int(r["Stream_Id"])
        if a.stream is not None and s != a.stream:
            continue
        b, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        out.append(((e - b) / 1e3, (b - t0) / 1e3, s, grid, short(r["Kernel_Name"])))
    if a.top:
        out = sorted(out, reverse=True)[: a.top]
    for d, st, s, g, n in out:
        print(f"{st:9.1f} {d:8.1f} us  s{s} grid {g:6d}  {n}")


if __name__ == "__main__":
    main()
