#!/usr/bin/env python3
"""boundary_gaps.py KERNEL_TRACE_CSV -- the gaps of tools/experiments/kernel_boundary.hip's run
(rocprofv3 --kernel-trace -f csv): median idle time between a kernel's end and the next kernel's
start, per segment of the program's fixed launch sequence (development tool)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "k_tiny" in r["Kernel_Name"] or "k_write" in r["Kernel_Name"]]
R = 20
segs = [("tiny -> tiny", 2 * R)]
for mib in (1, 16, 64, 256, 1024):
    segs += [(f"w{mib} MiB -> tiny / tiny -> w", 2 * R), (f"w{mib} MiB nt -> tiny / tiny -> w", 2 * R)]
segs.append(("graph: w1024 -> tiny / tiny -> w", 40))
for v in ("plain", "ext stop (device-scope)", "ext stop (system-scope)", "ext start+stop"):
    segs.append((f"w256 -> w256, {v}", R))
i = 0
for name, n in segs:
    seg = rows[i:i + n]
    i += n
    a, b = [], []  # gap after a writer (or 1st tiny), gap after a tiny
    for x, y in zip(seg, seg[1:]):
        gap = (int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) / 1e3
        (a if "k_write" in x["Kernel_Name"] or name.startswith("tiny") else b).append(gap)
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seg if "k_write" in r["Kernel_Name"]]
    print(f"{name:36s} gap after writer {statistics.median(a) if a else 0:7.2f} us   after tiny "
          f"{statistics.median(b) if b else 0:7.2f} us   writer {statistics.median(dur) if dur else 0:8.1f} us")
