"""Print grid / workgroup / LDS and duration of the first launch of every matching kernel in a
rocprofv3 kernel trace (development: launch geometry checks).  usage: kernel_grid.py TRACE.csv
[substr ...]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[2:] or [""]
seen = {}
for r in rows:
    n = r["Kernel_Name"]
    if any(p in n for p in pats):
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = n[:110]
        if k not in seen:
            seen[k] = [r.get("Grid_Size"), r.get("Workgroup_Size"),
                       r.get("LDS_Block_Size", r.get("Lds_Size")), []]
        seen[k][3].append(d)
for k, (g, w, l, ds) in seen.items():
    ds = sorted(ds)
    print(f"{k}\n    grid {g} wg {w} lds {l} launches {len(ds)} median {ds[len(ds) // 2] / 1e3:.1f} us")
