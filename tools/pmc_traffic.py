#!/usr/bin/env python3
"""HBM traffic of the roofline kernel from two rocprofv3 --pmc passes.

    python tools/pmc_traffic.py gpurun_out/TAG_pmc_fetch gpurun_out/TAG_pmc_write TAG [KERNEL BENCH_JSON WINDOWS]

WINDOWS 0 (default): the ingest windows of the run, counted as its k_exact_chunk_owner dispatches.

Each pass is its own `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` run of the same bench
command (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: they cannot share a pass).  Both counters
are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the
bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is taken as is.

Algorithmic bytes of a k_radix_scatter launch = n records x (8 B key [+ 8 B value]) read +
the same written; n is recovered from the grid (4096-record tiles, 256 threads per tile), the
last tile's padding (< 4096 records) being the only approximation.

Any other KERNEL (e.g. k_histo_exact, the bench's dominant kernel): its algorithmic bytes per
launch are taken from the bench line of the same command (BENCH_JSON, roofline.kernels), which
counts them from the launch's own work; the PMC traffic is averaged over every
dispatch of that kernel.

Writes roofline_traffic.json (read by bench.py for `roofline.traffic`) and a copy under
profiles/TAG_pmc_traffic.json.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "k_radix_scatter"
TILE, BLOCK = 4096, 512  # k_radix_scatter: 8 waves per 4096-record tile


def read_pass(path, counter):
    """dispatch id -> (kernel name, grid size, value) for one counter."""
    out = {}
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % path)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != counter:
                    continue
                key = (f, r["Dispatch_Id"])
                name = r["Kernel_Name"]
                grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
                v = float(r["Counter_Value"])
                if key in out:  # one row per (dispatch, counter) normally; sum instances otherwise
                    out[key] = (name, grid, out[key][2] + v)
                else:
                    out[key] = (name, grid, v)
    return out


def other_kernel(fetch, write, kernel, bench_json, tag, windows):
    """every dispatch of the kernel's family in the PMC runs (k_histo_exact: the one-wave and
    four-wave ingest replays, not the flush's k_histo_exact_list), per window, over the bench's
    launches per step -- the same unit as its algorithmic bytes per launch"""
    with open(bench_json) as fh:
        line = [ln for ln in fh.read().splitlines() if ln.startswith("{")][-1]
    kern = {k["kernel"]: k for k in json.loads(line)["roofline"]["kernels"]}[kernel]
    fam = (kernel, "k_exact_long_stats") if kernel == "k_histo_exact" else (kernel,)
    match = lambda name: any(k in name for k in fam) and "_list" not in name
    if windows <= 0:  # one k_exact_chunk_owner per ingest window with exact replays
        windows = sum(1 for (name, _, _) in fetch.values() if "k_exact_chunk_owner" in name)
    fb = [v * 1024.0 for (name, _, v) in fetch.values() if match(name)]
    wb = [v * 1024.0 for (name, _, v) in write.values() if match(name)]
    if not fb or len(fb) != len(wb):
        raise SystemExit("dispatch mismatch: %d fetch vs %d write rows" % (len(fb), len(wb)))
    n = windows * kern["launches_per_step"]
    fetch_b, write_b = 2.0 * sum(fb), sum(wb)
    alg = kern["algorithmic_bytes_per_launch"]
    return {
        "kernel": kernel,
        "dispatches": len(fb),
        "windows": windows,
        "traffic_per_launch": (fetch_b + write_b) / n,
        "fetch_per_launch": fetch_b / n,
        "write_per_launch": write_b / n,
        "algorithmic_per_launch": alg,
        "traffic_over_algorithmic": (fetch_b + write_b) / n / alg,
        "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), WRITE_SIZE x1; KiB -> bytes",
        "source": "profiles/%s_pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; "
                  "algorithmic bytes per launch from the bench line of the same command)" % tag,
    }


def main():
    fetch_dir, write_dir, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = read_pass(fetch_dir, "FETCH_SIZE")
    write = read_pass(write_dir, "WRITE_SIZE")
    if len(sys.argv) > 5 and sys.argv[4] != KERNEL:
        res = other_kernel(fetch, write, sys.argv[4], sys.argv[5], tag, int(sys.argv[6]) if len(sys.argv) > 6 else 0)
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        for p in (os.path.join(root, "roofline_traffic.json"),
                  os.path.join(root, "profiles", "%s_pmc_traffic.json" % tag)):
            with open(p, "w") as fh:
                json.dump(res, fh, indent=1)
        print(json.dumps(res, indent=1))
        return

    def scatter(rows):
        per = defaultdict(list)
        for (_, _), (name, grid, v) in sorted(rows.items(), key=lambda kv: int(kv[0][1])):
            if KERNEL in name:
                hasb = "<true" in name  # k_radix_scatter<true, NW>: 16-byte records
                n = (grid // BLOCK) * TILE
                per["bytes"].append(v * 1024.0)
                per["alg"].append(n * (32.0 if hasb else 16.0))
        return per

    f, w = scatter(fetch), scatter(write)
    if not f["bytes"] or len(f["bytes"]) != len(w["bytes"]):
        raise SystemExit("dispatch mismatch: %d fetch vs %d write rows" % (len(f["bytes"]), len(w["bytes"])))
    n = len(f["bytes"])
    fetch_b = 2.0 * sum(f["bytes"])  # gfx950: FETCH_SIZE counts half of a wide streaming read
    write_b = sum(w["bytes"])
    alg_b = sum(f["alg"])
    res = {
        "kernel": KERNEL,
        "dispatches": n,
        "traffic_per_launch": (fetch_b + write_b) / n,
        "fetch_per_launch": fetch_b / n,
        "write_per_launch": write_b / n,
        "algorithmic_per_launch": alg_b / n,
        "traffic_over_algorithmic": (fetch_b + write_b) / alg_b,
        "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), WRITE_SIZE x1; KiB -> bytes",
        "source": "profiles/%s_pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes)"
                  % tag,
    }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "roofline_traffic.json"), os.path.join(root, "profiles", "%s_pmc_traffic.json" % tag)):
        with open(p, "w") as fh:
            json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
