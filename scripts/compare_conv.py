#!/usr/bin/env python3
"""Per-shape A/B of two scripts/bench_conv.py logs (CSV rows + the JSON summary line):

    python scripts/compare_conv.py A.log B.log [--col fwd_ms,dgrad_ms,wgrad_ms]

Prints each shape's times in A and B and the ratio B/A, then the count-weighted totals."""
import json
import sys


def load(path):
    rows, head, summ = {}, None, None
    for line in open(path):
        line = line.strip()
        if line.startswith("{"):
            summ = json.loads(line)
        elif line.startswith("C,H,W"):
            head = line.split(",")
        elif head and line and line[0].isdigit():
            v = line.split(",")
            rows[tuple(v[:8])] = dict(zip(head, v))
    return rows, summ


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    cols = ["fwd_ms", "dgrad_ms", "wgrad_ms"]
    for i, x in enumerate(sys.argv):
        if x == "--col":
            cols = sys.argv[i + 1].split(",")
    print("shape".ljust(28) + "".join(f"{c:>22}" for c in cols))
    tot = {c: [0.0, 0.0] for c in cols}
    for k, ra in a[0].items():
        rb = b[0].get(k)
        if rb is None:
            continue
        cnt = int(ra["count"])
        cells = []
        for c in cols:
            va, vb = float(ra.get(c, 0) or 0), float(rb.get(c, 0) or 0)
            tot[c][0] += va * cnt
            tot[c][1] += vb * cnt
            cells.append(f"{va:7.3f}->{vb:7.3f} {vb / va if va else 0:5.2f}")
        print(("x".join(k) + f" x{cnt}").ljust(28) + "".join(f"{s:>22}" for s in cells))
    print("total".ljust(28) + "".join(f"{tot[c][0]:8.3f}->{tot[c][1]:7.3f} {tot[c][1] / tot[c][0] if tot[c][0] else 0:5.2f}"
                                      for c in cols))


if __name__ == "__main__":
    main()
