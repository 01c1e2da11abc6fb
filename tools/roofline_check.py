#!/usr/bin/env python3
"""Cross-check of bench.py's roofline line against the rocprofv3 kernel trace of the same run.

bench.py times the scatter launches (k_radix_scatter + the counter/gauge k_part_scatter) of its
last --timing-steps steps with HIP events on the engine stream, every class serialised on that
stream.  This reads the trace of `rocprofv3 --kernel-trace ... -- python3 bench.py ...` (the
gpu_check.sh profile run: those timing steps are the run's last steps), takes the scatter
launches of the last N steps that move >= 1M records (the longest-first key orderings of a few
hundred thousand keys are not part of bench's count), and prints their mean duration beside
bench's mean per launch.
    python tools/roofline_check.py gpurun_out/TAG_prof gpurun_out/TAG_prof.log [N=2]
"""
import csv
import glob
import json
import os
import sys


def main(prof_dir, bench_json, nsteps=2):
    rows = []
    for f in glob.glob(os.path.join(prof_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_flush_set" in r["Kernel_Name"]]
    lo = ends[-nsteps - 1] + 1
    durs = []
    for r in rows[lo:ends[-1] + 1]:
        name = r["Kernel_Name"]
        if "k_radix_scatter" not in name and "k_part_scatter" not in name:
            continue
        grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
        per_tile = int(r.get("Workgroup_Size_X") or 512)
        if grid // per_tile * 4096 < (1 << 20):
            continue
        durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    with open(bench_json) as fh:  # the bench JSON line (alone, or the last one in a log)
        b = json.loads([ln for ln in fh if ln.startswith("{")][-1])["roofline"]
    bench_us = b["ms_per_step"] * 1e3 / b["launches_per_step"]
    trace_us = sum(durs) / len(durs)
    print("scatter launches in the last %d steps of the trace: %d (bench: %.0f per step)" %
          (nsteps, len(durs), b["launches_per_step"]))
    print("mean duration: trace %.1f us, bench HIP events %.1f us (ratio %.3f)" % (trace_us, bench_us,
                                                                                  trace_us / bench_us))
    print("achieved at the trace's mean: %.0f GB/s (bench: %.0f GB/s)" %
          (b["algorithmic_bytes_per_launch"] / (trace_us * 1e-6) / 1e9, b["achieved"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2)
