"""Wall time vs kernel time per V-cycle from a rocprofv3 kernel trace: cycles are delimited
by the coarse solve (dense_gemv_kernel, once per cycle).  Usage: cycle_gaps.py trace.csv"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if not r["Kernel_Name"].startswith("__amd_rocclr")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "dense_gemv_kernel" in r["Kernel_Name"]]
walls, busy, counts = [], [], []
for a, b in zip(marks[-12:-1], marks[-11:]):
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    walls.append((t1 - t0) / 1e3)
    busy.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3)
    counts.append(len(seg))
print(f"cycles {len(walls)}: kernels/cycle {counts[-1]}, wall {sum(walls)/len(walls):.1f} us, "
      f"kernel time {sum(busy)/len(busy):.1f} us, gaps {(sum(walls)-sum(busy))/len(walls):.1f} us")
# per-kernel gap before it (launch-to-launch idle), last cycle
seg = rows[marks[-2]:marks[-1]]
print(f"{'kernel':60s} {'wgs':>7s} {'us':>8s} {'gap_before':>10s}")
prev_end = None
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev_end) / 1e3 if prev_end else 0.0
    nm = r["Kernel_Name"].replace("void ", "").replace("amg::(anonymous namespace)::", "").split("(")[0]
    print(f"{nm[:60]:60s} {int(r['Grid_Size_X'])//max(1,int(r['Workgroup_Size_X'])):7d} {(e-s)/1e3:8.1f} {g:10.1f}")
    prev_end = e
