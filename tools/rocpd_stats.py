#!/usr/bin/env python3
"""rocpd_stats.py DB [CSV] -- per-kernel statistics from a rocprofv3 rocpd SQLite database
(what `--stats` writes as CSV when the output format is csv; a torchrun-launched command
leaves the database form).  Columns as rocprofv3's kernel_stats.csv."""
import csv
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    tabs = [r[0] for r in db.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    rows = db.execute(f"select s.display_name, d.end - d.start from {kd} d join {ks} s "
                      f"on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, dur in rows:
        agg.setdefault(name, []).append(dur)
    total = sum(sum(v) for v in agg.values()) or 1
    out = []
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append({"Name": name, "Calls": len(v), "TotalDurationNs": sum(v),
                    "AverageNs": sum(v) / len(v), "Percentage": 100.0 * sum(v) / total,
                    "MinNs": min(v), "MaxNs": max(v)})
    w = csv.DictWriter(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout,
                       fieldnames=list(out[0].keys()) if out else ["Name"])
    w.writeheader()
    w.writerows(out)


if __name__ == "__main__":
    main()
