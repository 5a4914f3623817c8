#!/usr/bin/env python3
"""sort_timeline.py KERNEL_TRACE_CSV [which [first]] -- one whole sampled-plan sort of a rocprofv3
`--kernel-trace -f csv` run as a timeline (development tool): every dispatch from a K1e
(k_est_sample) to the next one, with start / end offsets, duration and a short name, so two
streams' kernels that overlap show up side by side.  `which` picks the sort (default: the
median-length one of those whose K3r took >= 200 us, i.e. the 2^28-key sorts; -1 = that default).
`first` names the kernel that starts a sort (default k_est_sample; k_hist16 for the exact plan and
the distributed sender, whose timeline then runs through the select and the receive sort)."""
import csv
import re
import sys


def short(name):
    n = name.replace("void ", "").replace("gsort::", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\s+", "", n.split("(")[0])[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = sys.argv[3] if len(sys.argv) > 3 else "k_est_sample"
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    sorts = []
    for a, b in zip(starts, starts[1:] + [len(rows)]):
        seg = rows[a:b]
        big = [r for r in seg if "k_partition_res" in r["Kernel_Name"] and
               int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) >= 200e3 and
               "true, true, unsigned int" in r["Kernel_Name"]]
        if big:
            end = max(int(r["End_Timestamp"]) for r in seg if any(
                k in r["Kernel_Name"] for k in ("k_local_sort_e", "k_count_expand", "k_partition_res",
                                                "k_gather_sort")))
            seg = [r for r in seg if int(r["Start_Timestamp"]) <= end]
            sorts.append(seg)
    if not sorts:
        sys.exit("no 2^28-key sampled-plan sort in the trace")
    spans = sorted(range(len(sorts)), key=lambda i: int(sorts[i][-1]["End_Timestamp"]) -
                   int(sorts[i][0]["Start_Timestamp"]))
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    if which < 0:
        which = spans[len(spans) // 2]
    seg = sorts[which]
    t0 = int(seg[0]["Start_Timestamp"])
    tend = max(int(r["End_Timestamp"]) for r in seg)
    print(f"sort {which} of {len(sorts)}: span {(tend - t0) / 1e3:.1f} us "
          f"(spans: min {min(int(s[-1]['End_Timestamp']) - int(s[0]['Start_Timestamp']) for s in sorts) / 1e3:.1f})")
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:7.1f}  "
              f"grid {r.get('Grid_Size', '?'):>9}  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
