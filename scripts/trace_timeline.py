"""Main-stream kernel timeline of one step from a rocprofv3 kernel trace: start offset, duration,
family, grid, and the share of each kernel's lifetime during which a side-stream kernel was also
running -- which GEMMs time-slice CUs with the weight-gradient stream:
python scripts/trace_timeline.py run_kernel_trace.csv [main_stream]"""
import csv
import sys

sys.argv += [] if len(sys.argv) > 2 else ["0"]
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "stem_image_kernel" in r["Kernel_Name"]]
spans = [(int(rows[j]["Start_Timestamp"]) - int(rows[i]["Start_Timestamp"]), i, j) for i, j in zip(idx, idx[1:])]
med = sorted(sp for sp, _, _ in spans)[len(spans) // 2]
a, b = [(i, j) for sp, i, j in spans if sp < 1.5 * med][-1]
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
main = sys.argv[2]
side = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in step if r["Stream_Id"] != main]


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("pdt::", "")
    return n[:60]


prev_end = t0
for r in step:
    if r["Stream_Id"] != main:
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ov = {}
    for ss, se, sid in side:
        o = min(e, se) - max(s, ss)
        if o > 0:
            ov[sid] = ov.get(sid, 0) + o
    ovs = " ".join(f"s{k}:{100 * v / max(1, e - s):.0f}%" for k, v in sorted(ov.items()))
    print(f"{(s - t0) / 1000:8.1f} gap{(s - prev_end) / 1000:6.1f} {(e - s) / 1000:7.1f} us  grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):6d} lds {r['LDS_Block_Size']:>6} v{r['VGPR_Count']:>4} a{r['Accum_VGPR_Count']:>4}  {short(r['Kernel_Name'])}  {ovs}")
    prev_end = e
