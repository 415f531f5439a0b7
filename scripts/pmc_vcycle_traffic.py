"""Per-launch HBM traffic of every bench.py vcycle_kernels operation, from the rocprofv3
--pmc passes of scripts/pmc_vcycle.py (one pass per counter).

traffic = 2 x FETCH_SIZE + WRITE_SIZE (bytes; on gfx950 FETCH_SIZE counts half the bytes of
wide coalesced reads, MI355X_MICROARCH.md "HBM") summed over the kernels one operation
launches, averaged over its 3 launches.  The dispatch stream is cut at the marker kernels
(uniform_kernel on 1000 + 2 op / 1000 + 2 op + 1 workgroups: segment start / end).  FETCH_SIZE counts the L2's memory-side requests,
Infinity-Cache hits included: for an operator that fits the 256 MiB cache the figure is
L2-miss traffic, not HBM traffic.

usage: pmc_vcycle_traffic.py <prefix> <ops.json> <out.json>
  reads <prefix>_FETCH_SIZE/run_counter_collection.csv and <prefix>_WRITE_SIZE/..."""
import csv
import json
import sys
from collections import defaultdict


def segments(path, counter, nops):
    rows = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        rows[d]["name"] = r["Kernel_Name"]
        rows[d]["grid"] = int(r["Grid_Size"]) // int(r["Workgroup_Size"])
        rows[d][counter] = rows[d].get(counter, 0.0) + float(r["Counter_Value"])
    seg = [None] * nops  # op index -> {kernel: summed counter}
    cur = None
    for d in sorted(rows):
        r = rows[d]
        if "uniform_kernel" in r["name"] and 1000 <= r["grid"] < 1000 + 2 * nops:
            m = r["grid"] - 1000  # 2 op: segment start, 2 op + 1: segment end
            cur = m // 2 if m % 2 == 0 else None
            if cur is not None:
                seg[cur] = defaultdict(float)
            continue
        if cur is not None:
            k = r["name"].split("(amg::")[0].replace("void amg::(anonymous namespace)::", "")
            seg[cur][f"{k} [{r['grid']}]"] += r[counter]
    return seg


def main(prefix, ops_path, out):
    meta = json.load(open(ops_path))
    ops, L = meta["ops"], meta["launches_per_op"]
    f = segments(f"{prefix}_FETCH_SIZE/run_counter_collection.csv", "FETCH_SIZE", len(ops))
    w = segments(f"{prefix}_WRITE_SIZE/run_counter_collection.csv", "WRITE_SIZE", len(ops))
    res = []
    for i, op in enumerate(ops):
        fetch = sum(f[i].values()) * 1024 / L
        write = sum(w[i].values()) * 1024 / L
        traffic = 2 * fetch + write
        res.append(dict(op, fetch_size_bytes=fetch, write_size_bytes=write, traffic_bytes=traffic,
                        traffic_over_stored=round(traffic / op["stored_bytes"], 4),
                        kernels=sorted(f[i])))
    doc = {"grid": meta["grid"], "definition": "2 x FETCH_SIZE + WRITE_SIZE per launch, summed over the "
           "operation's kernels (separate rocprofv3 --pmc passes; Infinity-Cache hits counted)",
           "ops": res}
    json.dump(doc, open(out, "w"), indent=1)
    for r in res:
        print(f"L{r['level']} {r['op']:16s} stored {r['stored_bytes'] / 1e6:8.1f} MB  traffic "
              f"{r['traffic_bytes'] / 1e6:8.1f} MB  ratio {r['traffic_over_stored']:.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
