#!/usr/bin/env python3
"""Per-window kernel sums of a C5 leg traced by rocprofv3 (tools/gpu/run.sh c5prof / c5profvar).

The global engine's windows each start with one k_gob_count (the histo import's count pass);
the kernels from one to the next are that window's.  Prints each window's kernel count, the sum
of its kernel durations and its span, then the kernel table of the timed window (the second:
bench.py runs one untimed window first).

usage: python tools/c5_trace_windows.py <run_kernel_trace.csv> [bench json or log]
"""
import collections
import csv
import json
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_gob_count" in r["Kernel_Name"]]
    bounds = starts + [len(rows)]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print("window  kernels  sum_ms  span_ms")
    for w in range(len(starts)):
        seg = rows[bounds[w]:bounds[w + 1]]
        span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
        print("%6d  %7d  %6.1f  %7.1f" % (w, len(seg), sum(dur(r) for r in seg), span))
    if len(sys.argv) > 2:
        txt = open(sys.argv[2]).read()
        m = re.search(r'"phases_ms_synchronised": (\{[^}]*\})', txt)
        if m:
            ph = json.loads(m.group(1))
            print("bench phases_ms_synchronised (same run): %s, sum %.1f ms" % (ph, sum(ph.values())))
    if len(starts) > 1:
        seg = rows[bounds[1]:bounds[2]]
        tot = collections.defaultdict(float)
        calls = collections.Counter()
        for r in seg:
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            tot[k] += dur(r)
            calls[k] += 1
        print("\nwindow 1 (timed) kernels:")
        print("%9s %6s  %s" % ("total_ms", "calls", "kernel"))
        for k, t in sorted(tot.items(), key=lambda x: -x[1]):
            if t >= 0.05:
                print("%9.2f %6d  %s" % (t, calls[k], k))


if __name__ == "__main__":
    main()
