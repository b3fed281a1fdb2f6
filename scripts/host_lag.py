"""Host-vs-device lag per kernel of one step from a rocprofv3 --kernel-trace --hip-trace run:
python scripts/host_lag.py TRACE_DIR [marker]
For every kernel of the last typical step: when its launch API returned (host), when it started on
the GPU, and the slack between them.  Slack near zero on a kernel that starts after an idle gap
means the device waited for the host (host-issue bound there); a large slack means it was queued."""
import csv
import os
import sys

d = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "stem_image_kernel"
api = {r["Correlation_Id"]: r for r in csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv")))}
rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
spans = [(int(rows[j]["Start_Timestamp"]) - int(rows[i]["Start_Timestamp"]), i, j) for i, j in zip(idx, idx[1:])]
med = sorted(s for s, _, _ in spans)[len(spans) // 2]
a, b = [(i, j) for s, i, j in spans if s < 1.5 * med][-1]
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
prev_end = {}
n_host = 0
host_wait = 0.0
for r in step:
    q = r["Queue_Id"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ar = api.get(r["Correlation_Id"])
    launched = int(ar["End_Timestamp"]) if ar else None
    slack = (s - launched) / 1000 if launched else float("nan")
    gap = (s - prev_end[q]) / 1000 if q in prev_end else 0.0
    prev_end[q] = max(prev_end.get(q, 0), e)
    flag = ""
    if gap > 5 and slack < 30:
        flag = "  <-- host-bound"
        n_host += 1
        host_wait += gap
    print(f"{(s - t0) / 1000:9.1f} q{q} dur {(e - s) / 1000:7.1f} gap {gap:7.1f} launch {((launched or t0) - t0) / 1000:9.1f} "
          f"slack {slack:8.1f}  {r['Kernel_Name'][:60]}{flag}")
print(f"host-bound starts: {n_host}, queue idle before them {host_wait:.1f} us")
