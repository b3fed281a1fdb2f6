"""Every kernel call of the last full training step in issue order, with stream, duration,
grid and registers (rocprofv3 kernel trace): python scripts/step_calls.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
step = rows[a + 1:b + 1]
t0 = int(step[0]["Start_Timestamp"])
for r in step:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pdt::", "")
    if n.startswith("igemm"):
        n = n.replace("igemm_nt_kernel", "nt").replace("igemm_tn_kernel", "tn").replace(" ", "")
    else:
        n = n.split("<")[0]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    print(f"{(s - t0) / 1000:9.1f} {r['Stream_Id']:>2} {(e - s) / 1000:8.1f}us grid {g:6d}x{r['Grid_Size_Y']:>3} "
          f"wg {r['Workgroup_Size_X']:>3} vgpr {r['VGPR_Count']:>3} agpr {r['Accum_VGPR_Count']:>3} lds {r['LDS_Block_Size']:>6}  {n}")
