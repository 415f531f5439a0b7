"""Per-cycle kernel time by (kernel, workgroups) from a rocprofv3 kernel trace.

Usage: cycle_breakdown.py run_kernel_trace.csv CYCLES
Kernels launched at least CYCLES times are counted as V-cycle kernels, with
calls // CYCLES launches per cycle; runtime copies/fills (setup) are skipped. The bench's
roofline loop adds extra level-0 SpMV launches, which the integer division absorbs."""
import collections
import csv
import sys


def short_name(full):
    nm = full.replace("void ", "").replace("amg::(anonymous namespace)::", "").replace("amg::", "")
    return nm.split("(")[0]


def main(path, cycles):
    agg = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith("__amd_rocclr"):
            continue
        k = (short_name(r["Kernel_Name"])[:64],
             int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
        agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
    out = []
    for k, v in agg.items():
        if cnt[k] >= cycles:
            per_cycle = cnt[k] // cycles
            out.append((v / cnt[k] * per_cycle, k, per_cycle, v / cnt[k]))
    tot = sum(o[0] for o in out)
    print(f"{'kernel':64s} {'wgs':>7s} {'x/cycle':>7s} {'avg us':>8s} {'us/cycle':>9s} {'share':>6s}")
    for per, k, pc, avg in sorted(out, reverse=True):
        print(f"{k[0]:64s} {k[1]:7d} {pc:7d} {avg:8.1f} {per:9.1f} {100 * per / tot:5.1f}%")
    print(f"sum per cycle {tot:.1f} us  ({cycles} cycles in the trace)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 23)
