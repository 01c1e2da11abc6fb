#!/usr/bin/env python3
"""Per-step timeline from a rocprofv3 kernel trace (bench.py run): steps end at k_flush_set.
Prints, for one step, every kernel group per stream with its busy time and [first start ..
last end] relative to the step start -- where the streams overlap and where the GPU idles.
  tools/timeline.py run_kernel_trace.csv [step] [min_busy_us]"""
import csv
import sys
from collections import defaultdict


def main(path, step=1, min_us=30.0):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_flush_set" in r["Kernel_Name"]]
    lo, hi = (ends[step - 1] + 1 if step else 0), ends[step] + 1
    t0 = int(rows[ends[step - 1]]["End_Timestamp"]) if step else int(rows[0]["Start_Timestamp"])
    agg = defaultdict(lambda: [0, 0.0, 1e18, 0.0])
    for r in rows[lo:hi]:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        name = name.replace("void ", "").replace("vn::", "")
        a = agg[(r["Stream_Id"], name[:34])]
        a[0] += 1
        a[1] += e - s
        a[2] = min(a[2], s)
        a[3] = max(a[3], e)
    print("step %d: %.1f us from the previous flush's last kernel to this flush's last" %
          (step, max(a[3] for a in agg.values())))
    for (q, name), (n, busy, s, e) in sorted(agg.items(), key=lambda kv: kv[1][2]):
        if busy >= min_us:
            print("s%-2s %-34s n=%4d busy %8.1f  [%8.1f .. %8.1f]" % (q, name, n, busy, s, e))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1, float(sys.argv[3]) if len(sys.argv) > 3 else 30.0)
