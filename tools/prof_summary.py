#!/usr/bin/env python3
"""Per-kernel statistics (rocprofv3 --stats layout) from a rocprofv3 run.

Reads either the rocpd SQLite database (`run_results.db`) or a `*_kernel_trace.csv`, and
writes `Name,Calls,TotalDurationNs,AverageNs,Percentage,MinNs,MaxNs` sorted by total time.
    python tools/prof_summary.py gpurun_out/TAG_prof profiles/r01_TAG_kernel_stats.csv
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def durations(path):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) if os.path.isdir(path) else [path]
    dbs = [p for p in dbs if p.endswith(".db")]
    out = defaultdict(list)
    if dbs:
        for db in dbs:
            c = sqlite3.connect(db)
            for name, d in c.execute("select name, duration from kernels"):
                out[name].append(int(d))
        return out
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                out[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    d = durations(src)
    tot = sum(sum(v) for v in d.values()) or 1
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    with open(dst, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, v in rows:
            w.writerow([name, len(v), sum(v), "%.1f" % (sum(v) / len(v)), "%.2f" % (100.0 * sum(v) / tot),
                        min(v), max(v)])
    print("%d kernels, %.3f ms total -> %s" % (len(rows), tot / 1e6, dst))


if __name__ == "__main__":
    main()
