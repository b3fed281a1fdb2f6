#!/usr/bin/env python3
"""Achieved HBM bandwidth per kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python scripts/hbm_summary.py gpurun_out/pmc_s5c_fetch gpurun_out/pmc_s5c_write [steps]

Both counters are in KiB per dispatch.  Durations come from the FETCH pass (the counter
passes serialize dispatches, so they are per-kernel times, not the overlapped step).
Prints one row per kernel (template args kept): calls, ms, GB read, GB written, TB/s.

gfx950 caveat (measured): FETCH_SIZE weights the 128-byte read requests as 64 bytes, so it
reports HALF the read traffic of streaming kernels (the fused SGD over 25.6 M fp32 params reads
param + grad + momentum = 307 MB and FETCH_SIZE says 153 MB).  The ``TB/s x2rd`` column doubles
the reads, which is the right figure for kernels whose loads are 128-B lines (every bf16x8 /
fp32x4 streaming kernel here); the raw column is a strict lower bound.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"pdt::(\w+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:48]


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    agg = defaultdict(lambda: [0, 0.0, 0.0])  # calls, value KiB, duration ns
    seen = set()
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
        if (disp, counter) in seen:
            continue
        seen.add((disp, counter))
        a = agg[k]
        a[0] += 1
        a[1] += float(r["Counter_Value"])
        a[2] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return agg


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    steps = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
    fe, wr = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    rows = []
    for k, (n, kib, ns) in fe.items():
        wkib = wr.get(k, [0, 0.0, 0.0])[1]
        rd, wb = kib * 1024 / 1e9, wkib * 1024 / 1e9
        rows.append((ns, k, n, rd, wb))
    rows.sort(reverse=True)
    tot_ns = sum(r[0] for r in rows)
    print(f"# per step (over {steps:g} profiled steps); serialized dispatch times")
    print(f"{'ms/step':>8} {'calls':>6} {'GB rd':>7} {'GB wr':>7} {'TB/s':>6} {'x2rd':>6}  kernel")
    for ns, k, n, rd, wb in rows[:40]:
        bw = (rd + wb) / (ns * 1e-9) / 1e3 if ns else 0.0
        bw2 = (2 * rd + wb) / (ns * 1e-9) / 1e3 if ns else 0.0
        print(f"{ns / 1e6 / steps:8.3f} {n / steps:6.0f} {rd / steps:7.3f} {wb / steps:7.3f} {bw:6.2f} {bw2:6.2f}  {k}")
    trd = sum(r[3] for r in rows) / steps
    twb = sum(r[4] for r in rows) / steps
    print(f"total: {tot_ns / 1e6 / steps:.3f} ms/step kernel time, {trd:.2f} GB read + {twb:.2f} GB written "
          f"per step, {(trd + twb) / (tot_ns / steps * 1e-9) / 1e3:.2f} TB/s averaged over kernel time "
          f"({(2 * trd + twb) / (tot_ns / steps * 1e-9) / 1e3:.2f} with reads doubled)")


if __name__ == "__main__":
    main()
