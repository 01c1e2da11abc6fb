#!/usr/bin/env python3
"""Cross-check of bench.py's roofline table against the rocprofv3 kernel trace of the same run.

bench.py times its kernels over its last --timing-steps steps with HIP events on the engine
stream, every class serialised on that stream (the earlier, timed steps run the classes
concurrently on several streams, so their launches share the GPU and last longer).  This reads
the trace of `rocprofv3 --kernel-trace ... -- python3 bench.py ... --timing-steps N` (the timing
steps are the run's last steps: tools/gpu/r03_prof.sh), and for every row of the bench's
roofline.kernels prints the trace's time of the same launches (the bench's launch count of that
kernel, largest grids first) beside the bench's figure, and the roofline fraction at the trace's
time.  With an output path it also writes the per-kernel statistics of those N steps (rocprofv3
--stats layout) -- the summary the bench figures are compared with.
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
    launches = defaultdict(list)  # base kernel name -> [(duration ns, grid)]
    for r in rows[lo:ends[-1] + 1]:
        name = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        per[name].append(d)
        base = name.replace("(anonymous namespace)", "").split("(")[0].split("<")[0].split("::")[-1].split()[-1]
        key = "k_histo_exact" if base.startswith("k_histo_exact") else base
        launches[key].append((d, int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)))
    with open(bench_json) as fh:  # the bench JSON line (alone, or the last one in a log)
        b = json.loads([ln for ln in fh if ln.startswith("{")][-1])["roofline"]
    # every kernel row of the bench table: the trace's launches of that kernel (template and
    # variant suffixes included) in the same timing step(s) -- the bench's launch count of them, the
    # largest grids first (bench times the window's big launches; small sorts of key orders and the
    # split engine's own launches run beside them) -- against bench's HIP-event figure
    for row in b["kernels"]:
        kname = row["kernel"]
        nb = max(1, int(round(row["launches_per_step"])) * nsteps)
        ls = sorted(launches.get(kname, []), key=lambda x: -x[1])
        pick = ls[:nb]
        if row.get("trace_kernels"):  # a phase of several kernels: every launch of each ("a&b": both in the name)
            pick = [(d, 0) for name, v in per.items() for d in v
                    if any(all(tok in name for tok in pat.split("&")) for pat in row["trace_kernels"])]
            ls, nb = pick, len(pick)
        ms_trace = sum(d for d, _ in pick) / 1e6 / nsteps
        rest = sum(d for d, _ in ls[nb:]) / 1e6 / nsteps
        print("%-16s trace %.3f ms/step over its %d largest launches (+%.3f ms in %d others), bench %.3f ms/step: "
              "ratio %.3f; frac at the trace's time %.4f (bench %.4f)" %
              (kname, ms_trace, len(pick), rest, len(ls) - len(pick), row["ms_per_step"],
               ms_trace / row["ms_per_step"] if row["ms_per_step"] else float("nan"),
               row["algorithmic_bytes_per_launch"] * row["launches_per_step"] / (ms_trace * 1e-3) / 1e9 / 8000.0
               if ms_trace else float("nan"), row["frac"]))
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
