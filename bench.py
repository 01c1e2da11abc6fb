#!/usr/bin/env python3
"""Benchmark: samples aggregated/sec per flush at 1M keys (BASELINE.json), C3 workload.

One step = one flush window on this GPU: ingest a 100M-sample mixed DogStatsD-shaped batch
(counters / gauges / timers / sets over 1M keys, Zipf(1.0) popularity, already parsed and
resident in HBM) through the engine's C-ABI, then flush it (Counter/Gauge values, Histo
local stats + p50/p90/p99/p99.9, Set estimates copied back to pinned host memory).

Multi-GPU: one process per GPU; keys are sharded by veneur's FNV-1a digest % N (the worker
routing of server.go:655), every rank aggregates its own 100M-sample shard stream (weak
scaling, no data-path collective).  value = samples of all ranks / max-over-ranks time.

The CPU baseline (rank 0, N=1) times the oracle -- a C restatement of the Go worker path
(samplers + tdigest + axiomhq HLL), multi-threaded with veneur's key routing -- on the same
stream; its flushed values also give the full-scale parity check and the p99 rank error.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PCT = (0.5, 0.9, 0.99, 0.999)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(d):
    """16 B per counter/gauge/histo record (slot u32 + value f64 + rate f32),
    8 B + member bytes per set record, plus per-key state read+written once per flush
    (counter 8 B, gauge 16 B, histo 40 B of local stats; centroids and HLL state excluded
    here -- a lower bound)."""
    n_scalar = len(d["c_slot"]) + len(d["g_slot"]) + len(d["h_slot"])
    b = 16 * n_scalar + 8 * len(d["s_slot"]) + int(len(d["s_bytes"]))
    nc, ng, nh, ns = d["n_slots"]
    b += 2 * (8 * nc + 16 * ng + 40 * nh)
    return b


def rank_error_stats(d, slots, eng_q, ref_q):
    """|F(q_engine) - F(q_ref)| with F the exact weighted empirical CDF of the key's samples."""
    hs, hv = d["h_slot"], d["h_val"]
    hw = (1.0 / d["h_rate"].astype(np.float32)).astype(np.float64)
    o = np.lexsort((hv, hs))
    sv, ss, sw = hv[o], hs[o], hw[o]
    cw = np.cumsum(sw)
    lo = np.searchsorted(ss, slots, side="left")
    hi = np.searchsorted(ss, slots, side="right")
    errs = np.zeros((len(slots), len(PCT)))
    for j in range(len(slots)):
        a, b = lo[j], hi[j]
        base = cw[a - 1] if a > 0 else 0.0
        tot = cw[b - 1] - base
        seg = sv[a:b]
        for k in range(len(PCT)):
            fe = np.searchsorted(seg, eng_q[j, k], side="right")
            fr = np.searchsorted(seg, ref_q[j, k], side="right")
            Fe = ((cw[a + fe - 1] - base) / tot) if fe else 0.0
            Fr = ((cw[a + fr - 1] - base) / tot) if fr else 0.0
            errs[j, k] = abs(Fe - Fr)
    return errs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--samples", type=int, default=100_000_000, help="samples per rank per flush window")
    ap.add_argument("--batches", type=int, default=1, help="ingest calls per flush window")
    ap.add_argument("--seed", type=int, default=0x5EED0003)
    ap.add_argument("--exact-threshold", type=int, default=0,
                    help="t-digest samples per key and window replayed bit-exactly (0: engine default)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: min(16, cpus))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timing-steps", type=int, default=2, help="untimed steps with per-kernel HIP-event timing")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps (for rocprof runs)")
    ap.add_argument("--pcie-steps", type=int, default=2,
                    help="extra steps from host arrays (vn_ingest_host), reported as pcie_inclusive; 0: off")
    args = ap.parse_args()

    import veneur_amd as V
    import veneur_amd._abi as A
    from veneur_amd.dist import Group, env_world

    world, rank, local_rank = env_world()
    group = Group(backend="nccl", local_rank=local_rank)  # world 1: no process group

    # ---- synthetic C3 shard stream (host), then resident in HBM
    t0 = time.time()
    d = V.synth(seed=args.seed, n_keys=args.keys, zipf_s=1.0, mix=(0.4, 0.2, 0.25, 0.15), n_samples=args.samples,
                shard=rank, n_shards=world, member_universe=50_000_000, rate_half=0.05, rate_tenth=0.05)
    n_slots = d["n_slots"]
    counts = [len(d["c_slot"]), len(d["g_slot"]), len(d["h_slot"]), len(d["s_slot"])]
    log(rank, "[bench] shard %d/%d: %d samples over %s keys (c/g/h/s=%s), generated in %.1fs" %
        (rank, world, args.samples, n_slots, counts, time.time() - t0))

    per_batch = [(c + args.batches - 1) // args.batches for c in counts]
    eng = V.Engine(tuple(max(1, x) for x in n_slots), compression=100.0, percentiles=PCT,
                   max_batch_records=max(per_batch) + 1, max_batch_member_bytes=int(len(d["s_bytes"])) + 64,
                   device=local_rank, exact_threshold=args.exact_threshold)
    bufs = []

    def dev(a):
        b = V.DeviceBuffer(a, device=local_rank)
        bufs.append(b)
        return b.ptr.value

    batches = []
    for bi in range(args.batches):
        b = A.Batch()
        sl = [slice(counts[c] * bi // args.batches, counts[c] * (bi + 1) // args.batches) for c in range(4)]
        b.n_counter = sl[0].stop - sl[0].start
        b.counter_slot, b.counter_value, b.counter_rate = dev(d["c_slot"][sl[0]]), dev(d["c_val"][sl[0]]), \
            dev(d["c_rate"][sl[0]])
        b.n_gauge = sl[1].stop - sl[1].start
        b.gauge_slot, b.gauge_value = dev(d["g_slot"][sl[1]]), dev(d["g_val"][sl[1]])
        b.n_histo = sl[2].stop - sl[2].start
        b.histo_slot, b.histo_value, b.histo_rate = dev(d["h_slot"][sl[2]]), dev(d["h_val"][sl[2]]), \
            dev(d["h_rate"][sl[2]])
        b.n_set = sl[3].stop - sl[3].start
        off = d["s_off"][sl[3].start:sl[3].stop + 1].astype(np.int64)
        b.set_slot = dev(d["s_slot"][sl[3]])
        b.set_member_off = dev((off - off[0]).astype(np.uint32))
        b.set_member_bytes = dev(d["s_bytes"][off[0]:off[-1]])
        batches.append(b)

    def step():
        for b in batches:
            eng.ingest_device(b)
        return eng.flush_raw()

    def sync():
        A.lib.vn_device_synchronize(local_rank)

    def barrier():
        group.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    sync()
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = step()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    # PCIe-inclusive rate (never `value`): the same window handed over as pageable host arrays
    # through vn_ingest_host (host-side checks, pinned staging, H2D copies, then the same kernels)
    pcie = None
    if args.pcie_steps > 0 and world == 1 and args.batches == 1:
        hkw = dict(counters=(d["c_slot"], d["c_val"], d["c_rate"]), gauges=(d["g_slot"], d["g_val"]),
                   histos=(d["h_slot"], d["h_val"], d["h_rate"]), sets=(d["s_slot"], d["s_off"], d["s_bytes"]))
        eng.ingest(**hkw)
        eng.flush_raw()
        sync()
        tp = time.perf_counter()
        for _ in range(args.pcie_steps):
            eng.ingest(**hkw)
            last = eng.flush_raw()
        sync()
        pms = (time.perf_counter() - tp) * 1e3 / args.pcie_steps
        pcie = {"value": args.samples / (pms * 1e-3), "unit": "samples/s", "ms_per_step": pms,
                "path": "vn_ingest_host from pageable host arrays: host checks + pinned staging + H2D + kernels"}
    # per-kernel timing (HIP events on the engine's stream) from extra, untimed steps: with
    # timing on, the side-stream classes run serialised so every launch is measured alone
    eng.timing_enable(True)
    tim = []
    for _ in range(max(1, args.timing_steps)):
        last = step()  # every step flushes the same window: parity below reads the latest result
        tim.append(eng.timing())
    eng.timing_enable(False)
    for _ in range(args.profile_steps):
        last = step()
    elapsed = group.max(elapsed)                                  # max over ranks
    total_samples = group.sum(float(args.samples)) * args.steps  # every rank's shard stream
    ms_per_step = elapsed * 1e3 / args.steps
    value = total_samples / elapsed

    # ---- roofline of the dominant kernel: the LSD radix scatter (histo key grouping + hot-key
    # value sort, set key grouping), algorithmic bytes = read + write of every record per pass
    sc_ms = float(np.mean([t["ms_radix_scatter_total"] for t in tim]))
    sc_bytes = float(np.mean([t["radix_scatter_bytes"] for t in tim]))
    sc_launch = float(np.mean([t["radix_scatter_launches"] for t in tim]))
    achieved = (sc_bytes / (sc_ms * 1e-3)) / 1e9 if sc_ms > 0 else 0.0
    phase = {k: round(float(np.mean([t[k] for t in tim])), 4) for k in
             ("ms_ingest_counter", "ms_ingest_gauge", "ms_ingest_histo", "ms_ingest_set", "ms_flush")}
    traffic, traffic_src, traffic_ratio = None, None, None
    tf = os.path.join(ROOT, "roofline_traffic.json")  # tools/pmc_traffic.py, PMC passes of this same command
    if os.path.exists(tf) and sc_launch:
        with open(tf) as fh:
            tj = json.load(fh)
        # the PMC passes measure HBM bytes / algorithmic bytes over every scatter dispatch of their
        # run; scaled to this step's launches (whose mix of record counts it shares)
        traffic_ratio = tj["traffic_over_algorithmic"]
        traffic, traffic_src = traffic_ratio * sc_bytes / sc_launch, tj["source"]
    path_bytes = algorithmic_bytes(d)
    path_gbs = path_bytes / (ms_per_step * 1e-3) / 1e9

    result = {
        "metric": "samples aggregated/sec per flush at 1M keys (1/2/4/8 GPU); p99 rank error",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64/u64",
        "data": "synthetic (DogStatsD-shaped C3 stream, seeded, resident in HBM)",
        "config": {"workload": "C3 mixed counters/gauges/timers/sets, %d keys, %d samples/flush/GPU, Zipf(1.0)"
                               % (args.keys, args.samples),
                   "keys": args.keys, "samples_per_gpu": args.samples, "batches_per_flush": args.batches,
                   "percentiles": list(PCT), "compression": 100, "hll_precision": 14,
                   "parallelism": "key-sharded FNV %% %d" % world},
        "roofline": {"bound": "hbm", "kernel": "k_radix_scatter", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "bytes per launch (HBM, PMC FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_over_algorithmic": traffic_ratio, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": sc_bytes / sc_launch if sc_launch else None,
                     "launches_per_step": sc_launch, "ms_per_step": sc_ms},
        "path": {"algorithmic_bytes_per_step": path_bytes, "effective_GBs": path_gbs,
                 "frac_of_hbm_peak": path_gbs / HBM_PEAK_GBS,
                 "phase_ms_serialised": phase, "ms_per_step_serialised": round(sum(phase.values()), 4)},
        "pcie_inclusive": pcie,
    }

    # ---- CPU baseline + full-scale parity (rank 0, N=1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        streams = {k: d[k] for k in ("c_slot", "c_val", "c_rate", "g_slot", "g_val", "h_slot", "h_val", "h_rate",
                                     "s_slot", "s_off", "s_bytes")}
        secs, _, ref = oracle.baseline_run_full(threads, n_slots, streams, PCT)
        result["cpu_baseline"] = {"value": args.samples / secs, "unit": "samples/s", "cores": threads,
                                  "kind": "port", "seconds": secs,
                                  "sample": "the full C3 flush window above (%d samples); C restatement of the Go "
                                            "Worker.ProcessMetric + flush path, %d worker threads routed by key"
                                            % (args.samples, threads)}
        # parity of the last timed step's flush with the restated reference
        o = last
        npct = len(PCT)
        c_slot = np.ctypeslib.as_array(o.counter_slot, shape=(o.n_counter,)).copy()
        c_val = np.ctypeslib.as_array(o.counter_value, shape=(o.n_counter,)).copy()
        g_slot = np.ctypeslib.as_array(o.gauge_slot, shape=(o.n_gauge,)).copy()
        g_val = np.ctypeslib.as_array(o.gauge_value, shape=(o.n_gauge,)).copy()
        h_slot = np.ctypeslib.as_array(o.histo_slot, shape=(o.n_histo,)).copy()
        h_q = np.ctypeslib.as_array(o.histo_quantiles, shape=(o.n_histo * npct,)).copy().reshape(-1, npct)
        h_st = np.ctypeslib.as_array(o.histo_stats, shape=(o.n_histo * 8,)).copy().reshape(-1, 8)
        s_slot = np.ctypeslib.as_array(o.set_slot, shape=(o.n_set,)).copy()
        s_est = np.ctypeslib.as_array(o.set_estimate, shape=(o.n_set,)).copy()
        par = {
            "counters_bit_exact": bool(np.array_equal(c_slot, np.nonzero(ref["touched"][0])[0]) and
                                       np.array_equal(c_val, ref["counter"][c_slot])),
            "gauges_bit_exact": bool(np.array_equal(g_slot, np.nonzero(ref["touched"][1])[0]) and
                                     np.array_equal(g_val, ref["gauge"][g_slot])),
            "sets_bit_exact": bool(np.array_equal(s_slot, np.nonzero(ref["touched"][3])[0]) and
                                   np.array_equal(s_est, ref["set_est"][s_slot])),
        }
        rs = ref["histo_stats"][h_slot]
        par["histo_minmax_weight_exact"] = bool(np.array_equal(h_st[:, :3], rs[:, :3]))
        with np.errstate(divide="ignore", invalid="ignore"):
            rel = np.abs(h_st[:, 3:5] - rs[:, 3:5]) / np.abs(rs[:, 3:5])
        par["histo_sum_max_rel_err"] = float(np.nanmax(rel))
        t1 = time.time()
        errs = rank_error_stats(d, h_slot, h_q, ref["histo_q"][h_slot])
        par["rank_error_max"] = {("p%g" % (100 * p)): float(errs[:, k].max()) for k, p in enumerate(PCT)}
        par["rank_error_mean"] = {("p%g" % (100 * p)): float(errs[:, k].mean()) for k, p in enumerate(PCT)}
        par["quantiles_bit_exact_frac"] = float(np.mean(np.all(h_q == ref["histo_q"][h_slot], axis=1)))
        result["p99_rank_error"] = par["rank_error_max"]["p99"]
        result["parity"] = par
        log(rank, "[bench] parity checked in %.1fs" % (time.time() - t1))
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    for b in bufs:
        b.free()
    group.close()


if __name__ == "__main__":
    main()
