"""Per-dispatch FETCH_SIZE (x2 gfx950 wide-stream correction, MI355X_MICROARCH.md) and
duration from one rocprofv3 --pmc FETCH_SIZE pass: python scripts/pmc_fetch.py <csv>"""
import csv
import sys

seen = set()
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] != "FETCH_SIZE":
        continue
    name = r["Kernel_Name"].replace("amg::(anonymous namespace)::", "").split("(")[0]
    grid = int(r["Grid_Size"]) // int(r["Workgroup_Size"])
    key = (name, grid)
    if key in seen:
        continue
    seen.add(key)
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    mb = float(r["Counter_Value"]) / 1024.0
    print(f"{name:48s} grid={grid:7d} {us:9.1f}us FETCH={mb:9.1f}MB x2={2 * mb:9.1f}MB "
          f"vgpr={r.get('VGPR_Count', '?')} lds={r.get('LDS_Block_Size', '?')}")
