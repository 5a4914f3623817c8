#!/usr/bin/env python3
"""select_gaps.py KERNEL_TRACE_CSV -- the distributed radix's select phase in a rocprofv3
`--kernel-trace -f csv` run of tools/group_bench.py (development tool).

Per rank (one HIP stream each) and step: the window from the sender's last level-2 partition
(K3a into the packed u16 buffer) to the first copy of the key exchange (the first copy after
K15 k_meta_counts), the kernels inside it, and the device's idle gaps in it -- time in which NO
stream of the process ran a kernel (the ranks share one GPU, so a rank waiting for a peer at a
collective is not idle time of the device)."""
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"],
                  r["Kernel_Name"]) for r in rows), key=lambda x: x[0])
    streams = sorted({e[2] for e in ev})
    windows = []
    for s in streams:
        mine = [e for e in ev if e[2] == s]
        i = 0
        while i < len(mine):
            n = mine[i][3]
            if "k_partition_res<1024, 8, false, false, unsigned short, false" in n:
                t0 = mine[i][1]
                j, seen_meta = i + 1, False
                while j < len(mine):
                    if "k_meta_counts" in mine[j][3]:
                        seen_meta = True
                    elif seen_meta and "copyBuffer" in mine[j][3]:
                        break
                    j += 1
                if j < len(mine):
                    windows.append((s, t0, mine[j][0], [e[3] for e in mine[i + 1:j]]))
                i = j
            else:
                i += 1
    if not windows:
        sys.exit("no sender K3a -> exchange window found")
    busy = sorted((e[0], e[1]) for e in ev)
    spans, gaps_all = [], []
    for s, a, b, names in windows:
        # device idle inside [a, b): the complement of the union of every stream's kernels
        t, gaps = a, []
        for x, y in busy:
            if y <= t or x >= b:
                continue
            if x > t:
                gaps.append(x - t)
            t = max(t, y)
        if b > t:
            gaps.append(b - t)
        spans.append(b - a)
        gaps_all.append(max(gaps) if gaps else 0)
    print(f"{len(windows)} select windows over {len(streams)} streams")
    print(f"window (K3a end -> first exchange copy): median {statistics.median(spans) / 1e3:.1f} us, "
          f"max {max(spans) / 1e3:.1f} us")
    print(f"largest device-idle gap per window: median {statistics.median(gaps_all) / 1e3:.2f} us, "
          f"max {max(gaps_all) / 1e3:.2f} us; windows with a gap > 10 us: "
          f"{sum(g > 10e3 for g in gaps_all)} of {len(gaps_all)}")
    s, a, b, names = windows[len(windows) // 2]
    short = [n.split("(")[0].replace("void ", "").replace("gsort::", "")
             .replace("(anonymous namespace)::", "")[:48] for n in names]
    print("kernels in one window:", ", ".join(short))


if __name__ == "__main__":
    main()
