"""Summarise a rocprofv3 kernel-trace CSV: per (kernel, grid) average duration, and the
per-V-cycle time split of the last N cycles (kernels between consecutive dense_gemv calls)."""
import csv
import sys
from collections import defaultdict


def main(path, ncyc=10):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    agg = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].replace("amg::(anonymous namespace)::", "").split("(")[0]
        key = (name, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':45s} {'grid':>8s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s}")
    for (k, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:40]:
        print(f"{k[:45]:45s} {g:8d} {len(v):6d} {sum(v)/len(v):9.2f} {min(v):9.2f}")
    # cycle segmentation by the coarse dense solve
    idx = [i for i, r in enumerate(rows) if "dense_gemv" in r["Kernel_Name"]]
    if len(idx) > ncyc + 1:
        spans = []
        for a, b in zip(idx[-ncyc - 1:-1], idx[-ncyc:]):
            t0 = int(rows[a]["Start_Timestamp"]); t1 = int(rows[b]["Start_Timestamp"])
            busy = sum(int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"]) for i in range(a, b))
            spans.append(((t1 - t0) / 1e3, busy / 1e3, b - a))
        print("gemv-to-gemv spans (us wall, us busy, kernels):", spans[-3:])


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
