#!/usr/bin/env python3
"""pmc_summary.py DIR -- per-kernel summary of a profile_pmc.sh run (JSON on stdout).

For every kernel: dispatches, average duration (kernel trace) and the average of every PMC
counter per dispatch.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reports half the bytes of a coalesced streaming read, so the read
side is FETCH_SIZE * 1024 * 2.  The factor is checked on the level-3 tile count (K1:
k_seg_counts<.., false, ..> or k_tile_counts), which reads exactly 4 B per key once
(`fetch_check` = corrected bytes / known bytes, expected 1.00).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("gsort::", "")
    n = n.split("(")[0]
    return n[5:] if n.startswith("void ") else n


def counters(d):
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def stats(d):
    res = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            res[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    return res


def main(root):
    summary = {"kernels": {}}
    st = stats(os.path.join(root, "stats"))
    pmc = {}
    subs = sorted(d for d in os.listdir(root)
                  if d != "stats" and os.path.isdir(os.path.join(root, d)))
    for sub in subs:  # every counter pass (profile_pmc.sh, profile_pipes.sh)
        for k, cs in counters(os.path.join(root, sub)).items():
            for c, vals in cs.items():
                pmc.setdefault(k, {})[c] = sum(vals) / len(vals)
    for k in sorted(set(st) | set(pmc)):
        summary["kernels"][k] = {**st.get(k, {}), **pmc.get(k, {})}
    bench = os.path.join(root, "stats.json")
    n = None
    try:
        line = json.loads(open(bench).read().strip().splitlines()[-1])
        n = line["config"]["keys_per_gpu"]
        summary["bench"] = {"value": line["value"], "ms_per_step": line["ms_per_step"],
                            "config": line["config"]}
    except (OSError, ValueError, IndexError, KeyError):
        pass
    cal = summary["fetch_calibration"] = 2.0
    for k, v in summary["kernels"].items():
        if (k.startswith("k_tile_counts") or k.startswith("k_seg_counts<512, false")) \
                and n and v.get("FETCH_SIZE"):
            summary["fetch_check"] = v["FETCH_SIZE"] * 1024 * cal / (n * 4)
    for k, v in summary["kernels"].items():
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v and cal:
            v["hbm_read_bytes"] = v["FETCH_SIZE"] * 1024 * cal
            v["hbm_write_bytes"] = v["WRITE_SIZE"] * 1024
            v["hbm_bytes"] = v["hbm_read_bytes"] + v["hbm_write_bytes"]
            if v.get("avg_us"):
                v["hbm_GBps"] = v["hbm_bytes"] / (v["avg_us"] * 1e3)
        if "TCC_EA0_RDREQ_sum" in v and "TCC_EA0_RDREQ_DRAM_sum" in v:
            # requests the L2s sent to the fabric but not to this GPU's DRAM: peer GPUs (xGMI)
            # or host memory; ~0 for a kernel that only touches local HBM
            v["ea_rdreq_non_dram"] = v["TCC_EA0_RDREQ_sum"] - v["TCC_EA0_RDREQ_DRAM_sum"]
            v["ea_wrreq_non_dram"] = v.get("TCC_EA0_WRREQ_sum", 0.0) - \
                v.get("TCC_EA0_WRREQ_DRAM_sum", 0.0)
        if "GRBM_GUI_ACTIVE" in v and v.get("avg_us"):
            v["eff_clock_GHz"] = v["GRBM_GUI_ACTIVE"] / 8 / (v["avg_us"] * 1e3)
    json.dump(summary, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
