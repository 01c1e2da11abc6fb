#!/usr/bin/env python3
"""Cross-check of bench.py's roofline line against the rocprofv3 kernel trace of the same run.

bench.py times the scatter launches (k_radix_scatter) of its last --timing-steps steps with HIP
events on the engine stream, every class serialised on that stream (the earlier, timed steps run
the classes concurrently on four streams, so their launches share the GPU and last longer).
This reads the trace of `rocprofv3 --kernel-trace ... -- python3 bench.py ... --timing-steps N`
(gpu_check.sh's profile run: the timing steps are the run's last steps), takes the scatter
launches of those last N steps that move >= 1M records (the longest-first key orderings of a few
hundred thousand keys are not part of bench's count), and prints their mean duration beside
bench's mean per launch.  With an output path it also writes the per-kernel statistics of those
N steps (rocprofv3 --stats layout) -- the summary the bench figures are compared with.
    python tools/roofline_check.py gpurun_out/TAG_prof gpurun_out/TAG_prof.log [N [stats.csv]]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(prof_dir, bench_json, nsteps=1, stats_out=None):
    rows = []
    for f in glob.glob(os.path.join(prof_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_flush_set" in r["Kernel_Name"]]
    lo = ends[-nsteps - 1] + 1
    durs = []
    per = defaultdict(list)
    for r in rows[lo:ends[-1] + 1]:
        name = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        per[name].append(d)
        if "k_radix_scatter" not in name:
            continue
        grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
        per_tile = int(r.get("Workgroup_Size_X") or 512)
        if grid // per_tile * 4096 < (1 << 20):
            continue
        durs.append(d / 1e3)
    with open(bench_json) as fh:  # the bench JSON line (alone, or the last one in a log)
        b = json.loads([ln for ln in fh if ln.startswith("{")][-1])["roofline"]
    k = [x for x in b["kernels"] if x["kernel"] == "k_radix_scatter"][0]
    bench_us = k["ms_per_step"] * 1e3 / k["launches_per_step"]
    trace_us = sum(durs) / len(durs)
    print("scatter launches in the last %d (timing) steps of the trace: %d (bench: %.0f per step)" %
          (nsteps, len(durs), k["launches_per_step"]))
    print("mean duration: trace %.1f us, bench HIP events %.1f us (ratio %.3f)" % (trace_us, bench_us,
                                                                                  trace_us / bench_us))
    print("achieved at the trace's mean: %.0f GB/s (bench: %.0f GB/s)" %
          (k["algorithmic_bytes_per_launch"] / (trace_us * 1e-6) / 1e9, k["achieved"]))
    if stats_out:
        tot = sum(sum(v) for v in per.values())
        with open(stats_out, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1,
         sys.argv[4] if len(sys.argv) > 4 else None)
