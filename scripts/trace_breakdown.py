"""Per-step kernel time by stream and kernel family from a rocprofv3 kernel trace (the last full
step between two launches of the marker kernel -- the stem's image conversion, the first kernel of a
step; the per-bucket optimizer launches several SGD kernels per step):
python scripts/trace_breakdown.py run_kernel_trace.csv [marker]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "stem_image_kernel"
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
# the last marker pair whose span is not an outlier (the bench's checksum / diagnostic steps follow)
spans = [(int(rows[j]["Start_Timestamp"]) - int(rows[i]["Start_Timestamp"]), i, j) for i, j in zip(idx, idx[1:])]
med = sorted(sp for sp, _, _ in spans)[len(spans) // 2]
a, b = [(i, j) for sp, i, j in spans if sp < 1.5 * med][-1]
step = rows[a:b]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
print(f"step span {(t1 - t0) / 1000:.1f} us, {len(step)} kernels")


def family(n):
    n = n.split("(")[0].replace("void ", "").replace("pdt::", "")
    if "igemm_ntq_kernel" in n:  # <WM, WN, TMQ, TNQ, EPI, OP, PIPE>
        args = n.split("<")[1].split(">")[0].split(",")
        return f"ntq epi{args[4].strip()} op{args[5].strip() if len(args) > 5 else '0'}"
    for key in ("igemm_nt_kernel", "igemm_tn_kernel", "bn_bwd_apply", "bn_act_fwd", "bn_finalize",
                "bn_bwd_part", "bn_bwd_reduce", "quant", "pool_bn", "fc_gemm", "sgd", "pack"):
        if key in n:
            if key == "igemm_nt_kernel":
                args = n.split("<")[1].split(">")[0].split(",")
                op = args[7].strip() if len(args) > 7 else "0"
                epi = args[6].strip()
                return f"nt epi{epi} op{op}"
            return key
    return n[:40]


by = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    k = (r["Stream_Id"], family(r["Kernel_Name"]))
    by[k][0] += 1
    by[k][1] += d
tot = collections.defaultdict(float)
for (s, n), (c, d) in sorted(by.items(), key=lambda x: -x[1][1]):
    tot[s] += d
    print(f"stream {s:>2} {c:4d} calls {d:9.1f} us  {n}")
print({k: round(v, 1) for k, v in tot.items()})
