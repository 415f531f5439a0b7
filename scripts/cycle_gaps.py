"""Per-V-cycle wall time, GPU-busy time and the largest idle gap, from a rocprofv3 kernel-trace
database (rocpd sqlite).  Cycles are delimited by the coarsest level's dense solve (one
*gemv* dispatch per cycle).  usage: python scripts/cycle_gaps.py <results.db> [last_n]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 31
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end, duration from kernels order by start"))
    g = [i for i, r in enumerate(rows) if "gemv" in r[0].lower()][-last:]
    print(f"{len(rows)} dispatches, {len(g)} cycle delimiters (last {last})")
    for a, b in zip(g[:-1], g[1:]):
        seg = rows[a:b]
        wall = (rows[b][1] - rows[a][1]) / 1e3
        busy = sum(r[3] for r in seg) / 1e3
        gaps = [(seg[i + 1][1] - seg[i][2]) / 1e3 for i in range(len(seg) - 1)]
        mg = max(gaps)
        print(f"wall {wall:9.1f} us  busy {wall and busy:8.1f} us  kernels {len(seg):3d}  "
              f"max idle gap {mg:8.1f} us after {seg[gaps.index(mg)][0][:70]}")


if __name__ == "__main__":
    main()
