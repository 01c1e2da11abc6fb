#!/usr/bin/env python3
"""Per-window chain view of a rocprofv3 kernel trace of bench.py (windows in flight): for each
ingest (k_validate_batch4 launch) the next k_histo_exact_mwb on any stream -- the hottest key's
chain -- with the gap from the ingest's start to the chain's start and the chain's duration,
plus the GPU's busy fraction (union of kernel intervals) over the traced span.
  tools/chain_windows.py run_kernel_trace.csv"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows]
    ing = [x for x in iv if "k_validate_batch4" in x[2]]
    mwb = [x for x in iv if "k_histo_exact_mwb" in x[2]]
    t0 = iv[0][0]
    print("%8s %8s %10s %10s %10s %6s" % ("ingest@", "chain@", "gap_ms", "chain_ms", "end@", "stream"))
    used = set()
    for s, e, n, st in ing:
        c = next((m for m in mwb if m[0] >= s and m not in used), None)
        if c is None:
            continue
        used.add(c)
        print("%8.1f %8.1f %10.2f %10.2f %10.1f %6s" % ((s - t0) / 1e6, (c[0] - t0) / 1e6, (c[0] - s) / 1e6,
                                                        (c[1] - c[0]) / 1e6, (c[1] - t0) / 1e6, c[3]))
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = max(e for _, e, _, _ in iv) - t0
    print("kernels %d  span %.1f ms  busy (union) %.1f ms  (%.0f%%)" % (len(iv), span / 1e6, busy / 1e6, 100.0 * busy / span))


if __name__ == "__main__":
    main(sys.argv[1])
