"""Concurrency of one training step from a rocprofv3 kernel trace (the last full step between two
optimizer launches): how long the GPU ran 0 / 1 / 2+ kernels, the idle gaps, and which kernels ran
alone longest.  Used to compare eager issue with HIP-graph replay, where every kernel may come
back on one queue and only the timestamps show whether the weight-gradient branch overlapped.

    python scripts/trace_overlap.py run_kernel_trace.csv [top_n]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
step = rows[a + 1:b + 1]
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in step]
t0 = min(s for s, _, _ in iv)
t1 = max(e for _, e, _ in iv)
ev = []
for s, e, _ in iv:
    ev.append((s, 1))
    ev.append((e, -1))
ev.sort()
hist = collections.defaultdict(float)
gaps = []
cur, last = 0, t0
for t, d in ev:
    if t > last:
        hist[min(cur, 3)] += (t - last) / 1000
        if cur == 0:
            gaps.append((t - last) / 1000)
    cur += d
    last = t
queues = collections.Counter(r.get("Queue_Id", r.get("Stream_Id", "?")) for _, _, r in iv)
print(f"step span {(t1 - t0) / 1000:.1f} us, {len(step)} kernels, queues {dict(queues)}")
print("time with 0/1/2/3+ kernels running (us): " +
      " ".join(f"{k}:{hist[k]:.1f}" for k in range(4)))
gaps.sort(reverse=True)
print(f"idle gaps: {len(gaps)}, total {sum(gaps):.1f} us, largest {[round(g, 1) for g in gaps[:8]]}")
# time each kernel family ran with nothing else on the GPU (sweep over start/end events)
alone = collections.defaultdict(float)
evk = sorted([(s, 1, i) for i, (s, _, _) in enumerate(iv)] + [(e, -1, i) for i, (_, e, _) in enumerate(iv)])
active, last = set(), t0
for t, d, i in evk:
    if t > last and len(active) == 1:
        (j,) = tuple(active)
        alone[iv[j][2]["Kernel_Name"].split("(")[0].replace("void ", "")[:60]] += (t - last) / 1000
    last = t
    (active.add if d > 0 else active.discard)(i)
print("kernels running alone longest (us):")
for k, v in sorted(alone.items(), key=lambda x: -x[1])[:top]:
    print(f"  {v:9.1f}  {k}")
