"""Per-cycle kernel time by (kernel, grid) from a rocprofv3 kernel trace: kernels that ran a
multiple of the cycle count (calls // cycles per V-cycle), sorted by time per cycle."""
import collections
import csv
import sys


def main(path, cycles):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in rows:
        nm = r["Kernel_Name"].split("(")[0]
        nm = nm.replace("void ", "").replace("amg::(anonymous namespace)::", "")
        k = (nm[:60], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
        agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
    tot = 0.0
    out = []
    for k, v in agg.items():
        if cnt[k] >= cycles:
            per = v / cnt[k] * (cnt[k] // cycles)
            tot += per
            out.append((per, k, cnt[k], v / cnt[k]))
    for per, k, c, avg in sorted(out, reverse=True):
        print(f"{k[0]:60s} {k[1]:8d} calls {c:5d} avg {avg:8.1f} us  per-cycle {per:8.1f} us")
    print(f"sum per cycle {tot:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 55)
