#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter CSVs per (short) kernel name: mean value per dispatch."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"pdt::(\w+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main(root):
    out = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        shape = os.path.basename(os.path.dirname(f)).rsplit("_s", 1)[0]
        for r in csv.DictReader(open(f)):
            if "pdt::" not in r["Kernel_Name"]:
                continue
            key = (shape, short(r["Kernel_Name"]))
            out[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            out[key]["_dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
            out[key]["_vgpr"].append(float(r["VGPR_Count"]) + float(r["Accum_VGPR_Count"]))
            out[key]["_lds"].append(float(r["LDS_Block_Size"]))
    for key in sorted(out):
        d = out[key]
        vals = {k: sum(v) / len(v) for k, v in d.items()}
        print(f"== {key[0]}  {key[1]}")
        print("   " + "  ".join(f"{k}={v:.4g}" for k, v in sorted(vals.items())))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
