#!/usr/bin/env python3
"""Per-kernel SQ counter ratios of a profiled training step (rocprofv3 --pmc, one pass).

    python scripts/sq_summary.py gpurun_out/pmc_s5h_sq [steps]

Columns: ms/step (serialized dispatches), waves, MFMA instructions, VALU instructions per MFMA
instruction (loader / epilogue issue overhead; the CDNA4 budget is about 2 per 16x16x32 MFMA),
MFMA-busy cycles as a share of CU-busy cycles, and wait cycles as a share of active-instruction
cycles.  The two shares are raw counter ratios (units as the counters define them), useful for
comparing kernels with each other, not as absolute utilisation.
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


def main():
    d = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = defaultdict(lambda: defaultdict(float))
    durs = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        durs[k][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    rows = sorted(((sum(durs[k].values()), k) for k in agg), reverse=True)
    print(f"# per step over {steps:g} profiled steps; serialized dispatch times")
    print(f"{'ms/step':>8} {'calls':>6} {'MFMA/step':>10} {'VALU/MFMA':>9} {'mfma/busy':>9} {'wait/act':>8}  kernel")
    for ns, k in rows[:30]:
        a = agg[k]
        mf = a.get("SQ_INSTS_MFMA", 0.0)
        va = a.get("SQ_INSTS_VALU", 0.0)
        vpm = va / mf if mf else float("nan")
        mb = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / a["SQ_BUSY_CU_CYCLES"] if a.get("SQ_BUSY_CU_CYCLES") else 0.0
        wa = a.get("SQ_WAIT_INST_ANY", 0.0) / a["SQ_ACTIVE_INST_ANY"] if a.get("SQ_ACTIVE_INST_ANY") else 0.0
        print(f"{ns / 1e6 / steps:8.3f} {len(durs[k]) / steps:6.0f} {mf / steps:10.3g} {vpm:9.2f} {mb:9.2f} {wa:8.2f}  {k}")


if __name__ == "__main__":
    main()
