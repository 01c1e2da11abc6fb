#!/usr/bin/env python3
"""The C4 window's counter and gauge records alone, ingested through the engine with timing on.

    python tools/scalar_bench.py [--steps 10] [--classes cg] [--check]

Builds the bench's C4 stream in HBM (vn_synth_device, the same seed and shape as bench.py),
then ingests only its counter and/or gauge arrays K times (one window each, flushed) and
prints the engine's HIP-event phase times (ms_ingest_counter, ms_ingest_gauge) and their
algorithmic rates.  Under `rocprofv3 --kernel-trace --stats` or `--pmc` it isolates the scalar
kernels (k_part_count, k_part_scatter, k_counter_runs, k_scalar_agg, k_gauge_*) from the
histogram and set work.  --check compares one window's flushed counters and gauges with numpy
(wrapping int64 sums; the last write per key in arrival order).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--samples", type=int, default=1_000_000_000)
    ap.add_argument("--seed", type=int, default=0x5EED0004)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--classes", default="cg")
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    import veneur_amd as V
    from veneur_amd import _abi as A

    t0 = time.time()
    s = V.DeviceStream(args.seed, args.keys, args.samples, 0, 1)
    b = A.Batch()
    C.memmove(C.byref(b), C.byref(s.batch), C.sizeof(A.Batch))
    b.n_histo = 0
    b.n_set = 0
    if "c" not in args.classes:
        b.n_counter = 0
    if "g" not in args.classes:
        b.n_gauge = 0
    nc, ng = int(b.n_counter), int(b.n_gauge)
    print("[scalar] %d counter and %d gauge records, %s slots, generated in %.1fs"
          % (nc, ng, s.n_slots, time.time() - t0), flush=True)
    with V.Engine(tuple(max(1, x) for x in s.n_slots), max_batch_records=max(s.counts) + 1,
                  max_class_records=tuple(int(c) + 1 for c in s.counts),
                  max_batch_member_bytes=64) as e:
        e.timing_enable(True)
        tim = []
        for _ in range(args.steps):
            e.ingest_device(b)
            tim.append(e.timing())
            out = e.flush_raw()
        mc = float(np.median([t["ms_ingest_counter"] for t in tim]))
        mg = float(np.median([t["ms_ingest_gauge"] for t in tim]))
        res = {"counter_records": nc, "gauge_records": ng, "ms_counter": mc, "ms_gauge": mg,
               "counter_GBs_16B": 16.0 * nc / (mc * 1e-3) / 1e9 if mc else None,
               "gauge_GBs_12B": 12.0 * ng / (mg * 1e-3) / 1e9 if mg else None,
               "ms_counter_all": [round(t["ms_ingest_counter"], 3) for t in tim],
               "ms_gauge_all": [round(t["ms_ingest_gauge"], 3) for t in tim]}
        if args.check:
            e.timing_enable(False)
            e.ingest_device(b)
            f = e.flush()
            h = s.to_host()
            ok = {}
            if nc:
                inv = (1.0 / h["c_rate"].astype(np.float32)).astype(np.float32).astype(np.float64)
                contrib = (h["c_val"].astype(np.int64) * inv.astype(np.int64))
                exp = np.zeros(s.n_slots[0], np.int64)
                np.add.at(exp, h["c_slot"], contrib)
                got = np.zeros(s.n_slots[0], np.int64)
                got[f.counter_slot] = f.counter_value
                ok["counters_exact"] = bool(np.array_equal(got, exp))
            if ng:
                last = np.full(s.n_slots[1], -1, np.int64)
                last[h["g_slot"]] = np.arange(len(h["g_slot"]))  # numpy fancy assignment: last wins
                touched = last >= 0
                exp = h["g_val"][last[touched]]
                got = np.full(s.n_slots[1], np.nan)
                got[f.gauge_slot] = f.gauge_value
                ok["gauges_exact"] = bool(np.array_equal(got[touched].view(np.uint64), exp.view(np.uint64)))
            res["check"] = ok
        print(json.dumps(res), flush=True)
    s.free()


if __name__ == "__main__":
    main()
