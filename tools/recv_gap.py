#!/usr/bin/env python3
"""recv_gap.py RUN_PREFIX -- the host-induced gap in front of every receive sort of a
rocprofv3 --kernel-trace (-f csv) of the distributed sorts (development tool; VERDICT r5 item
3).  Per launching thread (one rank of an in-process group, or a rank's process) and per sort:
the first receive-sort kernel (k_gather_sort / k_count_expand) is due once both its inputs are
in -- the last exchange copy (__amd_rocclr_copyBuffer on the rank's main stream) before it and
the receive plan (k_publish, on either stream) -- and starts `gap` us after that.  With the HIP API trace
(RUN_PREFIX_hip_api_trace.csv, --hip-runtime-trace) the launch call is matched by correlation id:
`host` = how long after `due` the host had enqueued the launch (<= 0: queued in time, so the gap
is the GPU's -- on a shared-GPU emulation, the other ranks' kernels -- not the host's).  Prints
every sort and the distribution."""
import csv
import statistics
import sys

import os
pre = sys.argv[1]
rows = sorted(csv.DictReader(open(pre + "_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
api = {}
if os.path.exists(pre + "_hip_api_trace.csv"):
    for a in csv.DictReader(open(pre + "_hip_api_trace.csv")):
        api[a["Correlation_Id"]] = int(a["End_Timestamp"])
hosts = []
by_thread = {}
for r in rows:
    by_thread.setdefault(r["Thread_Id"], []).append(r)
gaps = []
for th, rs in sorted(by_thread.items()):
    main = None
    for i, r in enumerate(rs):
        n = r["Kernel_Name"]
        if "k_gather_sort" in n or "k_count_expand" in n:
            main = main or r["Stream_Id"]
            # the sort this launch belongs to: look back to this sort's publish
            pub = copy = None
            for q in reversed(rs[:i]):
                qn = q["Kernel_Name"]
                if "k_gather_sort" in qn or "k_count_expand" in qn:
                    break
                if pub is None and "k_publish" in qn:
                    pub = q
                if copy is None and "copyBuffer" in qn and q["Stream_Id"] == r["Stream_Id"]:
                    copy = q
                if "k_hist16" in qn:
                    break
            if pub is None:
                continue  # a later receive kernel of the same sort
            due = max(int(pub["End_Timestamp"]), int(copy["End_Timestamp"]) if copy else 0)
            g = (int(r["Start_Timestamp"]) - due) / 1e3
            gaps.append(g)
            hl = (api[r["Correlation_Id"]] - due) / 1e3 if r["Correlation_Id"] in api else None
            if hl is not None:
                hosts.append(hl)
            print(f"thread {th} stream {r['Stream_Id']}: receive sort starts {g:7.1f} us after "
                  f"its last input ({'copy' if copy and int(copy['End_Timestamp']) >= int(pub['End_Timestamp']) else 'plan'})"
                  + (f"; launch enqueued {hl:+8.1f} us from it" if hl is not None else ""))
if gaps:
    print(f"{len(gaps)} receive sorts: gap median {statistics.median(gaps):.1f} us, max {max(gaps):.1f} us, "
          f"> 10 us: {sum(g > 10 for g in gaps)}")
if hosts:
    late = [min(h, g) for h, g in zip(hosts, gaps)]  # host-induced part of each gap
    print(f"host-induced (launch enqueued after the inputs were in, capped by the gap): median "
          f"{statistics.median(late):.1f} us, max {max(late):.1f} us, > 10 us: {sum(x > 10 for x in late)}")
