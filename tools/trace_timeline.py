#!/usr/bin/env python3
"""trace_timeline.py KERNEL_TRACE_CSV [N] -- the last N dispatches of a rocprofv3
`--kernel-trace -f csv` run as a timeline: start offset, duration and the idle gap before each
kernel (development tool: where a sort's device time goes between its kernels)."""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[-60:]
        print(f"{(s - t0) / 1e3:10.2f} us  dur {(e - s) / 1e3:8.2f} us  gap {gap:8.2f} us  "
              f"grid {r.get('Grid_Size', '?'):>9}  {name}")
        prev_end = e


if __name__ == "__main__":
    main()
