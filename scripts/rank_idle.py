"""Per-V-cycle GPU time split of one rank from a rocprofv3 kernel-trace CSV (multi-rank
rehearsals): over the last N cycles (delimited by the coarse dense solve, one
*dense_gemv* dispatch per cycle), the wall time, the time the compute kernels cover (union of
their intervals), the time only RCCL kernels run (waiting on the wire), and the time nothing
runs -- the host launch / synchronisation gaps that graph replay is meant to remove.
usage: python scripts/rank_idle.py <kernel_trace.csv> [last_n]"""
import csv
import sys


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + (cur_e - cur_s if cur_e is not None else 0)


def main(path, last=8):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "dense_gemv" in r["Kernel_Name"]][-(last + 1):]
    out = []
    for a, b in zip(idx[:-1], idx[1:]):
        t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        seg = [(max(t0, int(r["Start_Timestamp"])), min(t1, int(r["End_Timestamp"])), "nccl" in r["Kernel_Name"].lower())
               for r in rows if int(r["End_Timestamp"]) > t0 and int(r["Start_Timestamp"]) < t1]
        comp = union([(s, e) for s, e, n in seg if not n])
        anyk = union([(s, e) for s, e, _ in seg])
        out.append(((t1 - t0) / 1e3, comp / 1e3, (anyk - comp) / 1e3, (t1 - t0 - anyk) / 1e3,
                    sum(1 for r in rows[a:b] if "nccl" not in r["Kernel_Name"].lower())))
    print(f"{'wall_us':>9s} {'compute_us':>10s} {'rccl_only_us':>12s} {'idle_us':>9s} {'kernels':>7s}")
    for w, c, n, i, k in out:
        print(f"{w:9.1f} {c:10.1f} {n:12.1f} {i:9.1f} {k:7d}")
    if out:
        m = [sum(v[j] for v in out) / len(out) for j in range(4)]
        print(f"mean: wall {m[0]:.1f} us, compute {m[1]:.1f}, rccl-only {m[2]:.1f}, idle {m[3]:.1f} "
              f"({100 * m[3] / m[0]:.1f} % of the cycle)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8)
