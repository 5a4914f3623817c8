#!/usr/bin/env python3
"""step_timeline.py RUN_DIR_PREFIX FIRST [which] -- one step of a rocprofv3 trace (kernel,
memory-copy and, when present, HIP runtime API rows; -f csv) as a timeline (development tool).
A step runs from one dispatch of kernel FIRST to the next; `which` picks it (default: the
median-length step of the last half).  Every idle gap of the GPU (no kernel or copy running)
longer than 3 us is printed with the HIP API calls the host was inside at the time."""
import csv
import os
import re
import statistics
import sys


def short(n):
    n = n.replace("void ", "").replace("gsort::", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\s+", "", n.split("(")[0])[:64]


def load(path):
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


def main():
    pre, first = sys.argv[1], sys.argv[2]
    ev = []
    for r in load(pre + "_kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    for r in load(pre + "_memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   "copy " + r.get("Direction", "?") + " " + r.get("Bytes", "?") + " B"))
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
           for r in load(pre + "_hip_api_trace.csv")]
    ev.sort()
    starts = [i for i, e in enumerate(ev) if first in e[2]]
    steps = [ev[a:b] for a, b in zip(starts, starts[1:])]
    if not steps:
        sys.exit("no step")
    half = steps[len(steps) // 2:]
    lens = [s[-1][0] - s[0][0] for s in half]
    which = int(sys.argv[3]) if len(sys.argv) > 3 else None
    st = half[sorted(range(len(half)), key=lambda i: lens[i])[len(half) // 2]] if which is None \
        else steps[which]
    t0 = st[0][0]
    print(f"{len(steps)} steps; step length median {statistics.median(lens) / 1e3:.1f} us "
          f"(min {min(lens) / 1e3:.1f})")
    busy = t0
    idle = 0.0
    for s, e, n in st:
        gap = (s - busy) / 1e3
        if gap > 3:
            idle += gap
            host = sorted({f for a, b, f in api if a < s and b > busy})
            print(f"      -- idle {gap:7.1f} us; host in: {', '.join(host)[:150]}")
        print(f"{(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:7.1f}  {n}")
        busy = max(busy, e)
    print(f"idle gaps > 3 us: {idle:.1f} us of {(busy - t0) / 1e3:.1f}")


main()
