"""Per-launch HBM traffic of the level-0 SpMV from the PMC passes of scripts/gpu_pmc.sh.

traffic = 2 x FETCH_SIZE + WRITE_SIZE (bytes; FETCH_SIZE reads half the bytes of wide
streaming loads on gfx950, MI355X_MICROARCH.md "HBM"), averaged over the SpMV launches of
the 7-pt 256^3 level-0 operator (by default the plain-CSR kernel csr_plain_kernel<0>).  Writes a JSON
that bench.py reports as roofline.traffic."""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(path):
    vals = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        vals[d][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"], int(r["Grid_Size"]) // int(r["Workgroup_Size"]))
    return vals, meta


def main(prefix, out, kernels=("csr_plain_kernel<0",)):
    f, meta = per_dispatch(f"{prefix}_FETCH_SIZE/run_counter_collection.csv")
    w, _ = per_dispatch(f"{prefix}_WRITE_SIZE/run_counter_collection.csv")
    # level-0 operator = first matrix in pmc_levels.py: its first 3 SpMV launches (the
    # row-template kernel where the operator is templated, else the CSR block kernel)
    spmv = [d for d in sorted(meta) if any(k in meta[d][0] for k in kernels)]
    ds = [d for d in spmv if meta[d] == meta[spmv[0]]][:3]
    fetch = sum(f[d]["FETCH_SIZE"] for d in ds) / len(ds) * 1024
    write = sum(w[d]["WRITE_SIZE"] for d in ds) / len(ds) * 1024
    res = {"kernel": meta[ds[0]][0].split("(amg::")[0], "grid": meta[ds[0]][1], "launches": len(ds),
           "fetch_size_bytes": fetch, "write_size_bytes": write,
           "traffic_bytes": 2 * fetch + write,
           "note": "2 x FETCH_SIZE + WRITE_SIZE per launch, separate rocprofv3 --pmc passes"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    # argv[3] (optional): comma-separated kernel-name prefixes (default: the plain-CSR SpMV,
    # the bench's roofline kernel; "tpl_march_kernel<0" for the default-format one)
    main(sys.argv[1], sys.argv[2], *([tuple(sys.argv[3].split(","))] if len(sys.argv) > 3 else []))
