"""Print every counter of one or more rocprofv3 --pmc CSVs per dispatch (kernel, grid, us),
averaged over dispatches of the same (kernel, grid).  Usage: pmc_generic.py csv [csv ...]"""
import csv
import sys
from collections import defaultdict


def main(paths):
    vals = defaultdict(lambda: defaultdict(list))
    names = []
    for p in paths:
        per = defaultdict(dict)
        meta = {}
        for r in csv.DictReader(open(p)):
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] = float(r["Counter_Value"])
            nm = r["Kernel_Name"].replace("amg::(anonymous namespace)::", "").replace("void ", "")
            nm = nm[:nm.find("(amg")] if "(amg" in nm else nm.split("(")[0]
            meta[d] = (nm[:44], int(r["Grid_Size"]) // int(r["Workgroup_Size"]),
                       (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for d, cs in per.items():
            k = meta[d][:2]
            vals[k]["us"].append(meta[d][2])
            for c, v in cs.items():
                vals[k][c].append(v)
                if c not in names:
                    names.append(c)
    print(f"{'kernel':44s} {'grid':>7s} {'us':>8s} " + " ".join(f"{n[:16]:>16s}" for n in names))
    for k in sorted(vals, key=lambda k: -sum(vals[k]["us"])):
        v = vals[k]
        avg = lambda c: sum(v[c]) / len(v[c]) if v.get(c) else float("nan")
        print(f"{k[0]:44s} {k[1]:7d} {avg('us'):8.1f} " + " ".join(f"{avg(n):16.4g}" for n in names))


if __name__ == "__main__":
    main(sys.argv[1:])
