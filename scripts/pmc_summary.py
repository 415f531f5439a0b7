"""Join rocprofv3 --pmc pass CSVs (FETCH_SIZE, WRITE_SIZE, TCC_HIT/MISS) per dispatch.

gfx950 corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE (KB) reports half the bytes of a
wide coalesced streaming read -> x2 for the streamed part; WRITE_SIZE (KB) is exact for
16-B stores and uncalibrated for our 8-B stores.  We print raw and x2-corrected reads."""
import csv
import sys
from collections import defaultdict


def load(path):
    out = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        out[d][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"].replace("amg::(anonymous namespace)::", "").split("(")[0],
                   int(r["Grid_Size"]) // int(r["Workgroup_Size"]),
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                   int(r["VGPR_Count"]), int(r["SGPR_Count"]), int(r["LDS_Block_Size"]))
    return out, meta


def main(prefix):
    f, meta = load(f"{prefix}_FETCH_SIZE/run_counter_collection.csv")
    w, _ = load(f"{prefix}_WRITE_SIZE/run_counter_collection.csv")
    h, _ = load(f"{prefix}_TCC_HIT_sum/run_counter_collection.csv")
    print(f"{'kernel':34s} {'grid':>7s} {'us':>8s} {'vgpr':>4s} {'lds':>6s} {'FETCH_MB':>9s} "
          f"{'x2_MB':>8s} {'WRITE_MB':>9s} {'L2hit%':>7s}")
    for d in sorted(meta):
        k, g, us, vg, sg, lds = meta[d]
        if "csr_block" not in k and "gs" not in k and "tpl" not in k:
            continue
        fe = f[d].get("FETCH_SIZE", 0) / 1024
        wr = w.get(d, {}).get("WRITE_SIZE", 0) / 1024
        hh = h.get(d, {})
        hit = hh.get("TCC_HIT_sum", 0)
        miss = hh.get("TCC_MISS_sum", 0)
        hr = 100 * hit / (hit + miss) if hit + miss else 0
        print(f"{k[:34]:34s} {g:7d} {us:8.1f} {vg:4d} {lds:6d} {fe:9.1f} {2*fe:8.1f} {wr:9.1f} {hr:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
