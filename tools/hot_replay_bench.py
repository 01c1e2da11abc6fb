#!/usr/bin/env python3
"""Latency of the exact replay on hot keys: one window of K keys x n samples each (lognormal,
rate 1), ingested from HBM and flushed; reports ms per window and us per merge of the longest
key (n / 42 merges back to back), in the default (exact) mode and, with --fast, the opt-in
geometric mode.  Checks the quantiles against the oracle (bit-exact in exact mode).

  python tools/hot_replay_bench.py --n 1000000 --keys 1
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--keys", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--cold-keys", type=int, default=0, help="extra short keys in the same batch")
    ap.add_argument("--cold-n", type=int, default=100, help="samples per short key")
    ap.add_argument("--rates", action="store_true", help="10%% of samples at rate 0.5 or 0.1 (C4's mix)")
    ap.add_argument("--engines", type=int, default=1,
                    help="D > 1: D engines take 4 * D windows in turn (host threads, veneur_amd.dist.InTurn); "
                         "reports ms per window of that run as well")
    ap.add_argument("--reserved-cus", type=int, default=0)
    a = ap.parse_args()
    import veneur_amd as V
    import veneur_amd._abi as A
    rng = np.random.default_rng(1)
    slot = np.concatenate([np.repeat(np.arange(a.keys, dtype=np.uint32), a.n),
                           np.repeat(np.arange(a.keys, a.keys + a.cold_keys, dtype=np.uint32), a.cold_n)])
    rng.shuffle(slot)
    val = rng.lognormal(np.log(50.0), 1.0, len(slot))
    rate = np.ones(len(slot), np.float32)
    if a.rates:
        u = rng.random(len(slot))
        rate = np.where(u < 0.05, np.float32(0.1), np.where(u < 0.1, np.float32(0.5), np.float32(1.0))).astype(np.float32)
    pct = (0.5, 0.9, 0.99, 0.999)
    bufs = [V.DeviceBuffer(slot), V.DeviceBuffer(val), V.DeviceBuffer(rate)]
    nk = a.keys + a.cold_keys
    with V.Engine((1, 1, nk, 1), percentiles=pct, max_batch_records=len(slot) + 1,
                  exact_threshold=32768 if a.fast else 0) as e:
        b = A.Batch()
        b.n_histo = len(slot)
        b.histo_slot, b.histo_value, b.histo_rate = (x.ptr.value for x in bufs)
        times = []
        for r in range(a.reps + 1):
            A.lib.vn_device_synchronize(0)
            t0 = time.perf_counter()
            e.ingest_device(b)
            f = e.flush()
            A.lib.vn_device_synchronize(0)
            times.append(time.perf_counter() - t0)
        ms = min(times[1:]) * 1e3
        gobs = None
        if not a.no_check:  # the whole digest of the longest keys (GobEncode, pending merged)
            e.ingest_device(b)
            gobs = e.export_histos(np.arange(min(a.keys, 4), dtype=np.uint32))
            e.flush()
    pipe_ms = None
    if a.engines > 1:
        from veneur_amd.dist import InTurn
        engs = [V.Engine((1, 1, nk, 1), percentiles=pct, max_batch_records=len(slot) + 1,
                         replay_reserved_cus=a.reserved_cus) for _ in range(a.engines)]
        b = A.Batch()
        b.n_histo = len(slot)
        b.histo_slot, b.histo_value, b.histo_rate = (x.ptr.value for x in bufs)

        def work(k, i, turn):
            with turn(i, 1):
                engs[k].ingest_device(b)
            return engs[k].flush_raw()

        pipe = InTurn(a.engines)
        pipe.run(a.engines, work)
        A.lib.vn_device_synchronize(0)
        nwin = 4 * a.engines
        t0 = time.perf_counter()
        pipe.run(nwin, work)
        A.lib.vn_device_synchronize(0)
        pipe_ms = (time.perf_counter() - t0) * 1e3 / nwin
        for x in engs:
            x.close()
    merges = a.n // 42
    out = {"mode": "fast" if a.fast else "exact", "keys": a.keys, "samples_per_key": a.n, "cold_keys": a.cold_keys,
           "rates": a.rates, "ms_window": ms,
           "us_per_merge_longest": ms * 1e3 / max(1, merges)}
    if pipe_ms is not None:
        out["engines"] = a.engines
        out["ms_per_window_engines_in_turn"] = pipe_ms
    if not a.no_check:
        import oracle
        w = oracle.Worker(1, 1, nk, 1)
        w.histo(slot, val, rate)
        oq = np.array([[w.histo_quantile(k, p) for p in pct] for k in range(nk)])
        out["quantiles_bit_exact"] = bool(np.array_equal(f.histo_quantiles, oq))
        out["digests_bit_exact"] = all(g == w.histo_gob(k) for k, g in enumerate(gobs))
    print(out, flush=True)


if __name__ == "__main__":
    main()
