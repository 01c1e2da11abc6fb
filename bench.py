#!/usr/bin/env python3
"""Benchmark: samples aggregated/sec per flush at 1M keys (BASELINE.json), workload C4.

C4: ONE global DogStatsD-shaped stream of 1e9 samples per flush window
(counters / gauges / timers / sets over 1M keys, Zipf(1.0) popularity, already parsed),
key-sharded over the N GPUs of one node by veneur's worker routing, FNV-1a digest % N
(server.go:655).  In the opt-in fast mode (or with --split) the hot keys are split: the counter /
timer / set keys whose window count passes a share of the per-GPU load are dealt round-robin over
every GPU by their window arrival index and combined on their owner at flush over RCCL
(include/veneur_amd.h "multi-GPU"); in the default exact mode every key stays on its owner -- the
window is bound by the hottest timer's sequential chain, which no split can shorten.  Every
rank generates the whole stream on its GPU and keeps its own records, so the N ranks together
hold exactly the one stream (strong scaling: the total work is fixed, N = 1 processes all 1e9).

One step = one flush window per rank: the split-key lists, vn_ingest of the rank's batch
(resident in HBM), vn_ingest_split of its split-key records, vn_flush (the split-key exchange,
then Counter/Gauge values, Histo local stats + p50/p90/p99/p99.9, Set estimates to pinned host
memory).  value = 1e9 samples x steps / the max over ranks of the timed region.

Rank 0 at N = 1 also times the CPU baseline -- the oracle, a C restatement of the Go Worker path
(samplers + tdigest + axiomhq HLL) on 16 host threads with veneur's key routing -- on the same
window, and checks the flush against it (counters / gauges / sets bit-exact, histo stats, p99
rank error).  At N > 1 the ranks check stream invariants instead (counter total, histo weight).
"""
import argparse
import json
import os
import sys
import time

# Every engine stream its own hardware queue (HIP's default is 4 per process): with two engines in
# turn there are ~14 streams, and streams sharing a queue run one after another, a 200 ms replay
# in front holding back the other window's work.  Set before HIP initialises.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PCT = (0.5, 0.9, 0.99, 0.999)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "samples aggregated/sec per flush at 1M keys (1/2/4/8 GPU); p99 rank error"


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def hot_keys(counts, scale, classes, thr_cs, thr_set, max_split, split_histos=False):
    """Top keys by window count above the class threshold (counters: a share of the per-GPU
    load; sets: also any key that would keep one workgroup busy for long).  Timers only in the
    opt-in fast mode: the default exact mode replays every merge of a key on its owner, so a
    split timer would only move its records there."""
    from veneur_amd.dist import hot_keys as pick
    thr = {0: thr_cs, 3: thr_set}
    if split_histos:
        thr[2] = thr_cs
    out = pick(counts.astype(np.float64) * scale, classes, thr, max_split)
    out.setdefault(2, np.zeros(0, np.uint32))
    return out


def split_thresholds(args, thr):
    """{class: min window count} of the classes that split (timers only in the fast mode)."""
    t = {0: thr, 3: min(thr, args.set_hot)}
    if args.exact_threshold > 0:
        t[2] = thr
    return t


def split_from_engine(e, key_of_slot, thresholds, ctrl, max_split, keep=None):
    """vn_hot_keys of the flushed window on every rank, mapped to key ids and summed over the
    ranks (a split key's records are dealt over all of them); per class the hottest max_split
    above the threshold (sorted ids).  keep: the split list in use -- its keys stay while above
    half the threshold (hysteresis: a strided count near the threshold must not flip the list)."""
    local = {}
    for c, t in thresholds.items():
        slots, counts = e.hot_keys(c, int(t / (2 * ctrl.world)) + 1, 16 * max_split)
        local[c] = list(zip(key_of_slot[c][slots].tolist(), counts.tolist()))
    split = {0: np.zeros(0, np.uint32), 2: np.zeros(0, np.uint32), 3: np.zeros(0, np.uint32)}
    tot = {c: {} for c in thresholds}
    for part in ctrl.gather_object(local):
        for c, items in part.items():
            for k, n in items:
                tot[c][k] = tot[c].get(k, 0) + n
    for c, d in tot.items():
        t = thresholds[c]
        kept = set() if keep is None else set(np.asarray(keep.get(c, [])).tolist())
        hot = [(k, n) for k, n in d.items() if n > t or (k in kept and n > t / 2)]
        top = sorted(hot, key=lambda kv: (-kv[1], kv[0]))[:max_split]
        split[c] = np.sort(np.array([k for k, _ in top], np.uint32))
    return split


def detect_split(args, V, ctrl, world, rank, local_rank, thr):
    """The split list from the engines' hot-key detector over one unsplit window of the stream
    on every rank (detection stride args.hot_stride)."""
    s0 = V.DeviceStream(args.seed, args.keys, args.samples, rank, world, device=local_rank, split=None)
    with V.Engine(tuple(max(1, x) for x in s0.n_slots), compression=100.0, percentiles=PCT,
                  max_batch_records=max(s0.counts) + 1, max_class_records=tuple(int(c) + 1 for c in s0.counts),
                  max_batch_member_bytes=s0.counts[3] * 11 + 64, device=local_rank,
                  exact_threshold=args.exact_threshold) as e0:
        e0.hot_detect(args.hot_stride)
        e0.ingest_device(s0.batch)
        e0.flush_raw()
        split = split_from_engine(e0, s0.key_of_slot, split_thresholds(args, thr), ctrl, args.max_split)
    s0.free()
    return split, {"source": "engine hot-key detector (vn_hot_keys) over one unsplit window",
                   "stride": args.hot_stride}


def key_classes(seed, n_keys, mix=(0.4, 0.2, 0.25, 0.15)):
    """Class of every key (the generators' draw: splitmix64 of the key id)."""
    k = np.arange(n_keys, dtype=np.uint64)
    x = np.uint64(seed) ^ (np.uint64(0xA5A5A5A5) + k * np.uint64(0x9E3779B97F4A7C15))
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    u = (x >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    cum = np.cumsum(np.asarray(mix) / sum(mix))
    return np.minimum(np.searchsorted(cum, u, side="right"), 3).astype(np.int64)


def rank_error_stats(d, slots, eng_q, ref_q):
    """|F(q_engine) - F(q_ref)| with F the exact weighted empirical CDF of the key's samples; and
    each side's distance from the exact quantile, |F(q) - p| (SURVEY §8(d) accuracy metrics)."""
    want = np.zeros(int(d["h_slot"].max()) + 1 if len(d["h_slot"]) else 1, bool)
    want[slots] = True
    m = want[d["h_slot"]]
    hs, hv = d["h_slot"][m], d["h_val"][m]
    hw = (np.float32(1.0) / d["h_rate"][m]).astype(np.float64)
    o = np.lexsort((hv, hs))
    sv, ss, sw = hv[o], hs[o], hw[o]
    cw = np.cumsum(sw)
    lo = np.searchsorted(ss, slots, side="left")
    hi = np.searchsorted(ss, slots, side="right")
    errs = np.zeros((len(slots), len(PCT)))
    acc_e = np.zeros((len(slots), len(PCT)))
    acc_r = np.zeros((len(slots), len(PCT)))
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
            acc_e[j, k] = abs(Fe - PCT[k])
            acc_r[j, k] = abs(Fr - PCT[k])
    return errs, acc_e, acc_r


def c5_owners(n_keys, typ, world):
    """Owner rank of each C5 key, digest % N of its name and type (newJSONMetricsByWorker,
    http.go:71-139, with the GPUs as the workers): key k of a class is "c5.<typ>.<k>"."""
    from veneur_amd.worker import MetricKey, metric_digest
    return np.array([metric_digest(MetricKey("c5.%s.%d" % (typ, k), typ, "")) % world for k in range(n_keys)],
                    np.int64)


def c5_leg(args, rank, world, ctrl, device):
    """C5 (BASELINE configs[4]): a global veneur merging every host's forwarded digests and
    sketches -- ImportMetric -> Histo.Combine / Set.Combine (worker.go:230-268) for each of
    `hosts` DISTINCT hosts x (histo_keys GobEncode()d digests + set_keys MarshalBinary()d
    sketches); every key arrives from every host.  Each host's local window (~100 timer samples
    per key, Lomax-sized sets; vn_synth_hosts_device) is generated, ingested and exported on the
    GPU in groups of c5_group hosts (one local engine per group); the payloads stay in HBM,
    concatenated host-major.  Over N GPUs every rank sees every host and keeps the payloads of
    the keys it owns (digest % N, c5_owners: each key on exactly one rank, no collective).  One
    window = ONE vn_import_histos_device and ONE vn_import_sets_device call over the rank's
    payloads, then vn_flush; the window time is the max over the ranks.  Parity on sampled keys
    against the restated Go (oracle Worker.ImportMetric of the same payloads in the same host
    order): digest weight/min/max exact, set estimates exact, quantiles bit-exact (the default
    exact mode) -- rank error over the imported centroids reported as well."""
    import ctypes as C

    import oracle
    import veneur_amd as V
    import veneur_amd._abi as A
    H, S, hosts, G = args.c5_histo_keys, args.c5_set_keys, args.c5_hosts, max(1, args.c5_group)
    own = {2: np.nonzero(c5_owners(H, "timer", world) == rank)[0],
           3: np.nonzero(c5_owners(S, "set", world) == rank)[0]}
    nown = {c: len(own[c]) for c in own}
    rng = np.random.default_rng(args.seed + 5 + rank)
    # sampled keys, as indices into the rank's owned keys
    kh = np.sort(rng.choice(nown[2], min(nown[2], max(1, args.c5_parity_keys // world)), replace=False)) \
        if nown[2] else np.zeros(0, np.int64)
    ks = np.sort(rng.choice(nown[3], min(nown[3], max(1, args.c5_parity_keys // world)), replace=False)) \
        if nown[3] else np.zeros(0, np.int64)
    t0 = time.time()
    parts = {2: [], 3: []}  # per group: (offsets, DeviceBuffer)
    par = {2: {int(k): [] for k in kh}, 3: {int(k): [] for k in ks}}  # sampled keys' payloads, host order
    n_samples = 0
    for h0 in range(0, hosts, G):
        g = min(G, hosts - h0)
        win = V.HostWindows(args.seed + 55, h0, g, H, S, device=device)
        n_samples += win.n_histo + win.n_set
        with V.Engine((1, 1, g * H, g * S), percentiles=PCT, max_batch_records=max(win.n_histo, win.n_set) + 1,
                      max_batch_member_bytes=64, device=device) as loc:
            loc.ingest_device(win.batch)
            for cls, nk, keys in ((2, H, kh), (3, S, ks)):
                # this rank's keys of every host of the group, host-major
                sl = (np.arange(g, dtype=np.uint32)[:, None] * np.uint32(nk) + own[cls][None, :].astype(np.uint32))
                off, buf, view = loc.export_device(cls, sl.ravel().astype(np.uint32))
                parts[cls].append((off, buf))
                for hh in range(g):
                    for k in keys:
                        i = hh * nown[cls] + int(k)
                        par[cls][int(k)].append(view[off[i]:off[i + 1]].tobytes())
            loc.flush_raw()
        win.free()
    dev = {}
    payload_bytes = 0
    for cls in (2, 3):
        total = sum(int(o[-1]) for o, _ in parts[cls])
        big = V.DeviceBuffer.empty(total, device=device)
        offs, base = [], 0
        for o, b in parts[cls]:
            if int(o[-1]):
                A.lib.vn_device_copy(device, C.c_void_p(big.ptr.value + base), b.ptr, int(o[-1]))
            offs.append(o[:-1] + base)
            base += int(o[-1])
            b.free()
        offs.append(np.array([base], np.uint64))
        off_all = np.concatenate(offs).astype(np.uint64)
        slots = np.tile(np.arange(nown[cls], dtype=np.uint32), hosts)
        dev[cls] = (V.DeviceBuffer(slots, device=device), V.DeviceBuffer(off_all, device=device), big, len(slots))
        payload_bytes += total
    A.lib.vn_device_synchronize(device)
    gen_s = time.time() - t0
    with V.Engine((1, 1, max(1, nown[2]), max(1, nown[3])), percentiles=PCT, max_batch_records=args.c5_batch,
                  device=device) as g:
        def window():
            for cls in (2, 3):
                sl, of, by, n = dev[cls]
                if n:
                    g.import_device(cls, sl.ptr.value, of.ptr.value, by.ptr.value, n)
            return g.flush_raw()
        window()
        A.lib.vn_device_synchronize(device)
        ctrl.barrier()
        tw = time.perf_counter()
        for _ in range(args.c5_windows):
            f = window()
        A.lib.vn_device_synchronize(device)
        ms_rank = (time.perf_counter() - tw) * 1e3 / args.c5_windows
        ctrl.barrier()
        ms = ctrl.max(ms_rank)
        # one more window, synchronised between its phases (the split only; not the headline)
        phases = {}
        tp = time.perf_counter()
        for cls, name in ((2, "import_histos"), (3, "import_sets")):
            sl, of, by, n = dev[cls]
            if n:
                g.import_device(cls, sl.ptr.value, of.ptr.value, by.ptr.value, n)
            A.lib.vn_device_synchronize(device)
            phases[name] = (time.perf_counter() - tp) * 1e3
            tp = time.perf_counter()
        f = g.flush_raw()
        A.lib.vn_device_synchronize(device)
        phases["flush"] = (time.perf_counter() - tp) * 1e3
        # one more window with the engine's kernel timing (HIP events, phases run one after another):
        # the replay's own kernel time, to set against a profiler's trace of the same leg
        g.timing_enable(True)
        g.import_counts(reset=True)
        window()
        tmg = g.timing()
        icnt = g.import_counts()
        g.timing_enable(False)
        kernel_ms = {k: round(float(tmg[k]), 2) for k in ("ms_import_decode", "ms_import_drain", "ms_histo_replay",
                                                          "ms_radix_scatter_total", "ms_flush")}
        hq = np.ctypeslib.as_array(f.histo_quantiles, shape=(f.n_histo * len(PCT),)).reshape(-1, len(PCT)).copy() \
            if f.n_histo else np.zeros((0, len(PCT)))
        hst = np.ctypeslib.as_array(f.histo_stats, shape=(f.n_histo * 8,)).reshape(-1, 8).copy() \
            if f.n_histo else np.zeros((0, 8))
        hsl = np.ctypeslib.as_array(f.histo_slot, shape=(f.n_histo,)).copy() if f.n_histo else np.zeros(0, np.uint32)
        ses = np.ctypeslib.as_array(f.set_estimate, shape=(f.n_set,)).copy() if f.n_set else np.zeros(0, np.uint64)
        ssl = np.ctypeslib.as_array(f.set_slot, shape=(f.n_set,)).copy() if f.n_set else np.zeros(0, np.uint32)
    for d in dev.values():
        for b in d[:3]:
            b.free()
    # parity on sampled keys: the restated Go import of the same payload sequence
    t1 = time.time()
    w = oracle.Worker(1, 1, max(1, len(kh)), max(1, len(ks)))
    pos = {int(s_): j for j, s_ in enumerate(hsl)}
    st_exact, bit_exact, rank_err, st_diff = True, True, 0.0, np.zeros(3)
    for i, k in enumerate(kh):
        ms_, ws_ = [], []
        for pl in par[2][int(k)]:
            assert w.import_histo(i, pl) == 0
            t = oracle.MergingDigest(100.0)
            t.gob_decode(pl)
            m_, w_ = t.centroids()
            ms_.append(m_)
            ws_.append(w_)
        j = pos[int(k)]
        ost = np.array(w.histo_stats(i))
        st_exact &= bool(np.array_equal(hst[j, [5, 6, 7]], ost[[5, 6, 7]]))
        st_diff = np.maximum(st_diff, np.abs(hst[j, [5, 6, 7]] - ost[[5, 6, 7]]))
        ref_q = [w.histo_quantile(i, p) for p in PCT]
        bit_exact &= bool(np.array_equal(hq[j], ref_q))
        m, wt = np.concatenate(ms_), np.concatenate(ws_)
        o = np.argsort(m, kind="stable")
        sv, cw = m[o], np.cumsum(wt[o])
        F = lambda q: cw[np.searchsorted(sv, q, side="right") - 1] / cw[-1] if np.searchsorted(sv, q, side="right") \
            else 0.0
        for a, r in zip(hq[j], ref_q):
            rank_err = max(rank_err, abs(F(a) - F(r)))
    for i, k in enumerate(ks):
        for pl in par[3][int(k)]:
            w.import_set(i, pl)
    spos = {int(s_): j for j, s_ in enumerate(ssl)}
    set_exact = all(int(ses[spos[int(k)]]) == w.set_estimate(i) for i, k in enumerate(ks))
    # SURVEY §8(d)'s C5 bytes: the decoded contributions (16 B per centroid, 8192 B per dense sketch,
    # 4 B per sparse code) plus the output state written once (per histo key 40 B of statistics and
    # 16 B per centroid, at most 160 at delta 100; per set key its 8192 registers or 4 B per code,
    # bounded here by the dense size)
    decoded_bytes = 16 * icnt["centroids"] + 8192 * icnt["dense_sets"] + 4 * icnt["sparse_codes"] + \
        nown[2] * (40 + 16 * 160) + nown[3] * 8192
    per_rank = ctrl.gather_object({"ms": ms_rank, "keys": [nown[2], nown[3]], "payload_bytes": payload_bytes,
                                   "decoded_bytes": decoded_bytes, "import_counts": icnt,
                                   "phases": phases, "checked": [len(kh), len(ks)], "st_exact": st_exact,
                                   "st_diff": st_diff.tolist(), "bit_exact": bit_exact, "rank_err": rank_err,
                                   "set_exact": bool(set_exact)})
    n_imp = hosts * (H + S)
    all_bytes = sum(r["payload_bytes"] for r in per_rank)
    dec_bytes = sum(r["decoded_bytes"] for r in per_rank)
    return {"config": "C5 global import: %d distinct hosts x (%d histo digests + %d set sketches), every key from "
                      "every host; host windows generated, ingested and exported on the GPU (%d local samples per "
                      "rank); payloads in HBM, each rank keeping its keys' (digest %% %d), ONE "
                      "vn_import_histos_device + ONE vn_import_sets_device call per rank, then vn_flush"
                      % (hosts, H, S, n_samples, world),
            "n_gpus": world, "imports_per_s": n_imp / (ms * 1e-3), "payload_GBs": all_bytes / (ms * 1e-3) / 1e9,
            "ms_per_window": ms, "windows": args.c5_windows, "payloads_per_window": n_imp,
            "phases_ms_synchronised": {k: round(v, 2) for k, v in per_rank[0]["phases"].items()},
            "kernel_ms_timing_mode_rank0": kernel_ms,
            "ranks": {"ms_per_window": [round(r["ms"], 2) for r in per_rank],
                      "histo_set_keys": [r["keys"] for r in per_rank]},
            "payload_bytes_per_window": all_bytes,
            "roofline": {"bound": "hbm", "achieved_GBs": dec_bytes / (ms * 1e-3) / 1e9 / world, "peak": HBM_PEAK_GBS,
                         "frac": dec_bytes / (ms * 1e-3) / 1e9 / world / HBM_PEAK_GBS, "unit": "GB/s",
                         "bytes": "SURVEY §8(d): decoded contributions (16 B per centroid, 8192 B per dense sketch, "
                                  "4 B per sparse code) + output state, per window",
                         "algorithmic_bytes_per_window": dec_bytes,
                         "import_counts_rank0": per_rank[0]["import_counts"]},
            "roofline_payload": {"bound": "hbm", "achieved_GBs": all_bytes / (ms * 1e-3) / 1e9 / world,
                                 "peak": HBM_PEAK_GBS, "frac": all_bytes / (ms * 1e-3) / 1e9 / world / HBM_PEAK_GBS,
                                 "unit": "encoded payload bytes per second per GPU over the window"},
            "generated_in_s": round(gen_s, 2), "parity_checked_in_s": round(time.time() - t1, 2),
            "parity": {"keys_checked": {"histo": int(sum(r["checked"][0] for r in per_rank)),
                                        "set": int(sum(r["checked"][1] for r in per_rank))},
                       "histo_weight_min_max_exact": all(r["st_exact"] for r in per_rank),
                       "histo_min_max_weight_absdiff": np.max([r["st_diff"] for r in per_rank], axis=0).tolist(),
                       "histo_quantiles_bit_exact": all(r["bit_exact"] for r in per_rank),
                       "histo_rank_error_max": max(r["rank_err"] for r in per_rank),
                       "set_estimates_exact": all(r["set_exact"] for r in per_rank)}}


def text_leg(args):
    """SURVEY §8(f) rank 1 on the device: DogStatsD text already in HBM -> vn_intake_process (parse,
    Upsert into the device key table, ProcessMetric staging, vn_ingest) -> vn_flush, one window of
    text_passes buffers of text_lines lines; plus the parse alone (vn_parse_dogstatsd_device)."""
    import ctypes as C

    import veneur_amd as V
    import veneur_amd._abi as A
    from tools.parse_bench import make_buffer
    from veneur_amd.intake import DeviceParser, Intake
    buf = make_buffer(args.text_lines, n_keys=args.text_keys)
    cap = 1 << max(10, (args.text_keys - 1).bit_length())
    with V.Engine((cap,) * 4, percentiles=PCT, max_batch_records=args.text_lines) as e:
        it = Intake(e, max_bytes=len(buf) + 1, max_lines=args.text_lines)
        try:
            A.lib.vn_copy_to_device(e.device, it.buf.ptr, C.c_char_p(buf), len(buf))
            stats = []

            def window():
                stats.clear()
                for _ in range(args.text_passes):
                    stats.append(it.process_resident(len(buf)))
                f = e.flush_raw()
                it.reset()
                return f
            window()
            A.lib.vn_device_synchronize(e.device)
            t0 = time.perf_counter()
            for _ in range(args.text_windows):
                f = window()
            A.lib.vn_device_synchronize(e.device)
            ms = (time.perf_counter() - t0) * 1e3 / args.text_windows
            processed = sum(s["processed"] for s in stats)
            ok = processed == args.text_lines * args.text_passes and f.samples_processed == processed
        finally:
            it.close()
    with DeviceParser(max_bytes=len(buf) + 1, max_lines=args.text_lines + 1) as p:
        A.lib.vn_copy_to_device(0, p.buf.ptr, C.c_char_p(buf), len(buf))
        p.parse_resident(len(buf))
        A.lib.vn_device_synchronize(0)
        t0 = time.perf_counter()
        for _ in range(5):
            p.parse_resident(len(buf))
        A.lib.vn_device_synchronize(0)
        pms = (time.perf_counter() - t0) * 1e3 / 5
    lines = args.text_lines * args.text_passes
    return {"config": "DogStatsD text in HBM: %d buffers of %d lines (%d bytes, %d keys, Zipf 1.3, 3 tags, C3 type "
                      "mix) per window -> vn_intake_process -> vn_flush" % (args.text_passes, args.text_lines, len(buf),
                                                                             args.text_keys),
            "lines_per_s": lines / (ms * 1e-3), "ms_per_window": ms, "text_GBs": len(buf) * args.text_passes /
            (ms * 1e-3) / 1e9, "parse_only_lines_per_s": args.text_lines / (pms * 1e-3),
            "parse_only_ms_per_buffer": pms, "new_keys_first_buffer": stats[0]["new_keys"] if stats else 0,
            "checks": {"every_line_processed": bool(ok)}}


def egress_leg(flush_result):
    """the C4 window's flush result -> InterMetrics -> Datadog request bodies
    (vn_datadog_flush, native), every touched key named "c4.<class>.<slot>" with two tags."""
    import veneur_amd._abi as A
    from veneur_amd.sink import DatadogSink
    from veneur_amd.worker import DEFAULT_AGGREGATES
    arr = lambda p, n: np.ctypeslib.as_array(p, shape=(n,)).copy() if n else np.zeros(0, np.uint32)
    parts = [(0, arr(flush_result.counter_slot, flush_result.n_counter), b"c"),
             (2, arr(flush_result.gauge_slot, flush_result.n_gauge), b"g"),
             (6, arr(flush_result.histo_slot, flush_result.n_histo), b"t"),
             (8, arr(flush_result.set_slot, flush_result.n_set), b"s")]
    mp, sl, names = [], [], []
    for m, slots, tag in parts:
        mp.append(np.full(len(slots), m, np.uint8))
        sl.append(slots.astype(np.uint32))
        names += [b"c4.%s.%d" % (tag, s) for s in slots.tolist()]
    tags = [b"env:prod,host:h%d" % (i % 100) for i in range(len(names))]
    blob = b"".join(n + t for n, t in zip(names, tags))
    nlen = np.array([len(n) for n in names], np.uint32)
    tlen = np.array([len(t) for t in tags], np.uint32)
    noff = np.zeros(len(names), np.uint64)
    if len(names):
        noff[1:] = np.cumsum(nlen.astype(np.uint64) + tlen)[:-1]
    mp, sl = np.concatenate(mp), np.concatenate(sl)
    nt = np.full(len(names), 2, np.uint32)
    bb = np.frombuffer(blob or b"\0", np.uint8)
    keys = A.Keys(len(names), mp.ctypes.data_as(A.u8p), sl.ctypes.data_as(A.u32p), nt.ctypes.data_as(A.u32p),
                  noff.ctypes.data_as(A.u64p), nlen.ctypes.data_as(A.u32p), tlen.ctypes.data_as(A.u32p),
                  bb.ctypes.data_as(A.u8p))
    sink = DatadogSink(10.0, "bench-host", ["dc:1"], 5000)
    try:
        import ctypes as C
        cfg = A.DDConfig()
        cfg.interval, cfg.timestamp, cfg.is_local, cfg.aggregates = 10.0, 1_700_000_000, 0, DEFAULT_AGGREGATES.value
        cfg.n_percentiles = len(PCT)
        for i, p in enumerate(PCT):
            cfg.percentiles[i] = p
        ep = np.array(PCT, np.float64)
        cfg.engine_percentiles = ep.ctypes.data_as(A.f64p)
        cfg.hostname, cfg.sink_tags, cfg.n_sink_tags, cfg.flush_max_per_body = b"bench-host", b"dc:1", 1, 5000
        out = A.DDPayload()
        t0 = time.perf_counter()
        rc = A.lib.vn_datadog_flush(sink.h, C.byref(flush_result), C.byref(keys), C.byref(cfg), C.byref(out))
        dt = time.perf_counter() - t0
        assert rc == 0
        nbytes = np.ctypeslib.as_array(out.body_off, shape=(out.n_bodies + 1,))[-1]
        ok = int(np.ctypeslib.as_array(out.body_status, shape=(out.n_bodies,)).tolist().count(0))
    finally:
        sink.close()
    return {"config": "the C4 window's flush result (%d keys) -> generateInterMetrics -> finalizeMetrics -> JSON "
                      "bodies of <= 5000 series (vn_datadog_flush, one host core)" % len(names),
            "intermetrics": int(out.n_intermetrics), "series": int(out.n_metrics), "bodies": int(out.n_bodies),
            "bodies_encoded": ok, "body_MB": float(nbytes) / 1e6, "ms": dt * 1e3,
            "intermetrics_per_s": out.n_intermetrics / dt}


def cgroup_cpus():
    """The cgroup v2 (cpu.max) or v1 (cfs quota / period) CPU limit of this process, rounded up;
    None when no limit is set or none can be read."""
    import math
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        if q != "max":
            return max(1, math.ceil(int(q) / int(p)))
        return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            p = int(fh.read())
        return max(1, math.ceil(q / p)) if q > 0 else None
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)  # ~1.3 s timed at C4: long enough for SMI sampling
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--samples", type=int, default=1_000_000_000, help="samples per flush window, all ranks")
    ap.add_argument("--seed", type=int, default=0x5EED0004)
    ap.add_argument("--hot-div", type=int, default=32,
                    help="split a counter/timer key above samples / (N * hot_div) per window")
    ap.add_argument("--set-hot", type=int, default=1 << 18, help="split a set key above this many records")
    ap.add_argument("--max-split", type=int, default=64, help="split keys per class at most")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="engines per GPU taking the windows in turn (window i + 1 ingested and combined while "
                         "window i's longest replays finish; one communicator per engine, the combines entered in "
                         "window order); 1: one engine, windows back to back; 0 (default): 5 at N = 1, 7 beyond (the whole "
                         "C4 bench at N = 1: 60.2 / 56.9 / 56.4 ms per window at 4 / 5 / 6 engines, the C5 leg beside six "
                         "slower, 166 against 142 ms; the hottest key's rank at N = 2 / 4 / 8 35.6 / 31.0 / 29.0 ms with "
                         "7 engines against 52.4 / 47.9 / 45.7 with 4, DESIGN.md §6)")
    ap.add_argument("--reserved-cus", type=int, default=0,
                    help="CUs kept for the longest exact replays (vn_config.replay_reserved_cus); 0 (default): none")
    ap.add_argument("--no-stagger", dest="stagger", action="store_false",
                    help="D > 1: let the engines' ingests start together (default: in window order)")
    ap.add_argument("--hot-stride", type=int, default=256,
                    help="hot-key detector: count every hot_stride-th record (vn_hot_detect)")
    ap.add_argument("--no-split", action="store_true", help="route every key by digest %% N (no hot keys)")
    ap.add_argument("--split", action="store_true",
                    help="exact mode: split the hot counter / set keys as the fast mode does (default: off -- "
                         "measured, DESIGN.md §6: the window is bound by the hottest timer's chain, which a "
                         "split cannot shorten, and the combine costs every rank more than the balance gains)")
    ap.add_argument("--exact-threshold", type=int, default=0,
                    help="0 (default): every histogram merge replayed exactly; N: the opt-in fast mode "
                         "(geometric pieces past N samples per key, rank-error parity only)")
    ap.add_argument("--hot-prefix", type=int, default=0,
                    help="exact window prefix of keys past 4x the exact threshold (0: the engine's default)")
    ap.add_argument("--piece-growth", type=int, default=0, help="geometric piece growth in %% (0: default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: min(16, cpus))")
    ap.add_argument("--parity-keys", type=int, default=3000, help="histo keys sampled for the rank-error check")
    ap.add_argument("--timing-steps", type=int, default=1,
                    help="untimed steps with per-kernel HIP-event timing (0: none)")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps (for rocprof runs)")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="development only: run rank --sim-rank's share of an N-GPU split on this one GPU "
                         "(no exchange partners; not a bench result)")
    ap.add_argument("--sim-rank", type=int, default=0)
    ap.add_argument("--c5-hosts", type=int, default=1000, help="C5 leg (rank 0, N=1): hosts per window (0: off)")
    ap.add_argument("--c5-histo-keys", type=int, default=10000)
    ap.add_argument("--c5-set-keys", type=int, default=2000)
    ap.add_argument("--c5-group", type=int, default=50, help="hosts generated per local engine")
    ap.add_argument("--c5-batch", type=int, default=64 << 20, help="the global engine's max_batch_records")
    ap.add_argument("--c5-windows", type=int, default=1)
    ap.add_argument("--c5-parity-keys", type=int, default=256)
    ap.add_argument("--text-lines", type=int, default=2_000_000,
                    help="DogStatsD text intake leg (rank 0, N=1): lines per buffer (0: off)")
    ap.add_argument("--text-passes", type=int, default=8, help="buffers per intake window")
    ap.add_argument("--text-keys", type=int, default=100_000)
    ap.add_argument("--text-windows", type=int, default=2)
    ap.add_argument("--split-delay-ms", type=float, default=0.0, help="development only: host delay after split_close")
    ap.add_argument("--host-trace", action="store_true",
                    help="development only: report host ms in split_keys+ingest_split / ingest / flush")
    ap.add_argument("--worker-windows", type=int, default=-1,
                    help="windows of the Worker-level leg (veneur_amd.Worker over the same D engines: Flush "
                         "hands the window's engine to its flush thread and ingest moves to the next one); "
                         "-1 (default): --steps, 0: off")
    ap.add_argument("--c5-only", action="store_true", help="run the C5 leg alone (for its rocprof trace)")
    ap.add_argument("--pcie-steps", type=int, default=1,
                    help="extra steps from host arrays (vn_ingest_host), reported as pcie_inclusive; 0: off")
    args = ap.parse_args()

    import veneur_amd as V
    import ctypes as C

    import veneur_amd._abi as A
    from veneur_amd.dist import Group, InTurn, env_world, make_comm

    world, rank, local_rank = env_world()
    sim = args.sim_world > 1 and world == 1
    ctrl = Group(backend="gloo")  # host control plane: barrier, max / sum of scalars, the RCCL id
    if args.c5_only:
        c5 = c5_leg(args, rank, world, ctrl, local_rank)
        if rank == 0:
            print(json.dumps({"c5": c5}), flush=True)
        ctrl.close()
        return
    comm = make_comm(ctrl, local_rank)  # the engines' RCCL group (None at N = 1)

    # ---- hot keys: chosen by the engines' own detector (vn_hot_detect / vn_hot_keys) from a
    # window they have seen -- one unsplit window of the stream, every rank counting its share,
    # the ranks' candidates summed by key (the --sim-world development mode, which sees one
    # rank's share only, keeps the count of the stream's first 2^24 records)
    t0 = time.time()
    split = {0: np.zeros(0, np.uint32), 2: np.zeros(0, np.uint32), 3: np.zeros(0, np.uint32)}
    detect = None
    # hot keys split over the GPUs: the fast mode's default; in the exact mode only with --split
    if args.exact_threshold == 0 and not args.split:
        args.no_split = True
    if not args.no_split:
        thr = args.samples / ((args.sim_world if sim else world) * args.hot_div)
        if sim:
            sample = min(args.samples, 1 << 24)
            counts = V.synth_key_counts(args.seed, args.keys, args.samples, sample, device=local_rank)
            split = hot_keys(counts, args.samples / sample, key_classes(args.seed, args.keys), thr,
                             min(thr, args.set_hot), args.max_split, split_histos=args.exact_threshold > 0)
        else:
            split, detect = detect_split(args, V, ctrl, world, rank, local_rank, thr)
    stream = V.DeviceStream(args.seed, args.keys, args.samples, args.sim_rank if sim else rank,
                            args.sim_world if sim else world, device=local_rank, split=split)
    n_slots = stream.n_slots
    log(rank, "[bench] rank %d/%d: %d of %d samples (c/g/h/s=%s, split h/s=%s), %s slots, split keys c/h/s=%s, "
        "generated in %.1fs" % (rank, world, stream.n_records, args.samples, list(stream.counts),
                                list(stream.split_counts), n_slots, [len(split[c]) for c in (0, 2, 3)],
                                time.time() - t0))

    # D engines take the windows in turn (window i on engine i % D), each driven by its own host
    # thread: window i + 1 is ingested while window i's longest replays finish -- as the
    # reference's flush goroutine works on the swapped maps while the workers take the next
    # interval.  Flushes are entered in window order, so every rank issues the split combine's
    # collectives (one communicator per engine) in the same order.
    nw = args.sim_world if sim else world
    D = max(1, args.pipeline if args.pipeline > 0 else (5 if nw <= 1 else 7))

    # (measured, DESIGN.md §4: the reservation costs the other windows more than it gains)
    reserved = max(0, args.reserved_cus)

    def make_engine():
        e = V.Engine(tuple(max(1, x) for x in n_slots), compression=100.0, percentiles=PCT,
                     max_batch_records=max(stream.counts) + 1,
                     max_class_records=tuple(int(c) + 1 for c in stream.counts),
                     max_batch_member_bytes=stream.counts[3] * 11 + 64, device=local_rank,
                     exact_threshold=args.exact_threshold, hot_prefix=args.hot_prefix,
                     piece_growth=args.piece_growth, split_max_records=max(stream.split_counts) + 1,
                     replay_reserved_cus=reserved)
        if detect is not None:
            e.hot_detect(args.hot_stride)  # the live detector keeps counting inside the timed steps
        return e

    engines = [make_engine() for _ in range(D)]
    eng = engines[0]
    if comm is not None:
        eng.set_comm(comm)
        for e in engines[1:]:
            e.set_comm(make_comm(ctrl, local_rank))
    split_lists = []
    for c in (0, 2, 3):
        slots = (stream.split_slot0[c] + np.arange(len(split[c]))).astype(np.uint32)
        owners = (stream.digest_of_slot[c][slots] % np.uint32(world)).astype(np.uint32)
        split_lists.append((c, slots, owners))

    host_marks = []  # --host-trace: host clock at each call's return (development)
    pipe = InTurn(D)
    lat = []  # per window: host ms from its first call to its flush's return
    ing = []  # per window: host ms from its first call to its ingest's return (the ingest's own syncs included)

    import contextlib

    def step(k=0, i=None, turn=None):
        e = engines[k]
        # the ingests in window order (D > 1): the engines' long replays, which start as an
        # ingest ends, follow one another instead of all starting together
        gate = turn(i, 1) if (turn is not None and D > 1 and args.stagger) else contextlib.nullcontext()
        t = [time.perf_counter()] if args.host_trace and D == 1 else None
        ts = time.perf_counter()
        with gate:
            for c, slots, owners in split_lists:
                if len(slots):
                    e.split_keys(c, slots, owners)
            # split records first: they are buffered on the split engine's stream, so the split
            # combine at flush does not wait behind this engine's ingest
            if sum(stream.split_counts):
                e.ingest_split_device(stream.split)
                if D == 1:
                    e.split_close()  # their combine runs beside this engine's ingest
                if args.split_delay_ms:
                    time.sleep(args.split_delay_ms * 1e-3)
            if t:
                t.append(time.perf_counter())
            e.ingest_device(stream.batch)
        ing.append((time.perf_counter() - ts) * 1e3)
        if t:
            t.append(time.perf_counter())
        if turn is not None and D > 1:
            # only the split combine's collectives need the window order (one communicator per
            # engine, every rank issuing them in the same order); the replays and the flush of
            # window i then run beside window i + 1's ingest and combine on the other engines
            with turn(i):
                e.split_combine()
        r = e.flush_raw()
        lat.append((time.perf_counter() - ts) * 1e3)
        if t:
            t.append(time.perf_counter())
            tm = e.timing()
            host_marks.append(np.concatenate([np.diff(t) * 1e3, [tm["ms_split_host"], tm["ms_main_ready"],
                                                                 tm["ms_split_ready"], tm["ms_split_histo_ready"],
                                                                 tm["ms_split_set_prefix_ready"]]]))
        return r

    def run_windows(n):
        """n windows; returns the last one's flush result."""
        return pipe.run(n, step)[-1] if n else None

    def sync():
        A.lib.vn_device_synchronize(local_rank)

    # every engine's first window sizes its scratch (hipMalloc / hipFree: a hipFree waits for the
    # whole device, the other engines' replays included), so each engine warms up at least once
    warm = max(args.warmup, D)
    run_windows(warm)
    sync()
    # the profiling build (VN_LIB=libveneur_amd_prof.so): the batched replay's phase cycles of each
    # window's longest key (block 0), summed over the timed windows (tools/exact_profile.py's fields)
    prof_read = getattr(A.lib, "vn_prof_exact_read", None)
    prof_buf = None
    if prof_read is not None:
        prof_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
        prof_buf = (C.c_ulonglong * 64)()
        prof_read(prof_buf, 1)
    ctrl.barrier()
    lat.clear()
    ing.clear()
    t0 = time.perf_counter()
    last = run_windows(args.steps)
    sync()
    t_rank = time.perf_counter() - t0
    exact_prof = None
    if prof_buf is not None:
        prof_read(prof_buf, 0)
        pv = list(prof_buf)
        nb = max(1, pv[23])
        exact_prof = {"batches": pv[23], "avg_committed": round(pv[24] / nb, 2), "avg_usable": round(pv[26] / nb, 2),
                      "avg_flagged": round(pv[25] / nb, 2), "structural": pv[22],
                      "avg_repairs": round(pv[32] / nb, 2), "cyc_repair": round(pv[33] / nb, 1),
                      "cyc_batch_call": round(pv[27] / nb, 1)}
        for i, nme in zip((16, 17, 18, 19, 15, 20, 21, 48, 13), ("totals", "A", "B", "C", "D", "E_C2", "F", "G", "H")):
            exact_prof["cyc_" + nme] = round(pv[i] / nb, 1)
        exact_prof["cyc_E_per_wave"] = [round(pv[36 + w] / nb, 1) for w in range(4)]
        exact_prof["cyc_C2_per_wave"] = [round(pv[44 + w] / nb, 1) for w in range(4)]
    ctrl.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = ctrl.max(elapsed)
    rank_ms = ctrl.gather_object(t_rank * 1e3 / args.steps)
    window_latency_ms = ctrl.max(float(np.mean(lat))) if lat else None
    window_ingest_ms = ctrl.max(float(np.mean(ing))) if ing else None
    last_eng = engines[(args.steps - 1) % D]
    if host_marks:
        log(rank, "[bench] host ms per call (split+ingest_split, ingest, flush; split combine in flush); device ms to main / split ready / split histos / set prefix: %s" %
            np.round(np.mean(host_marks[args.warmup:] or host_marks, axis=0), 3).tolist())
    if detect is not None:
        # the split list the detector picks from the last timed window: the one in use
        redetect = split_from_engine(last_eng, stream.key_of_slot, split_thresholds(args, thr), ctrl,
                                     args.max_split, keep=split)
        detect["stable_over_timed_windows"] = all(np.array_equal(redetect[c], split[c]) for c in split)
    rank_records = ctrl.gather_object(stream.n_records)
    ms_per_step = elapsed * 1e3 / args.steps
    value = float(args.samples) * args.steps / elapsed

    # stream invariants of the flushed window (all ranks): counter total, histo weight
    fc = np.ctypeslib.as_array(last.counter_value, shape=(last.n_counter,)).astype(np.int64) if last.n_counter \
        else np.zeros(0, np.int64)
    hst = np.ctypeslib.as_array(last.histo_stats, shape=(last.n_histo * 8,)).reshape(-1, 8) if last.n_histo \
        else np.zeros((0, 8))
    with np.errstate(over="ignore"):
        csum_flushed = int(fc.sum(dtype=np.int64))
    inv = ctrl.gather_object((csum_flushed, stream.counter_sum, float(hst[:, 0].sum()), stream.histo_weight))
    wrap = lambda v: (v + (1 << 63)) % (1 << 64) - (1 << 63)
    checks = {"counter_total_exact": wrap(sum(i[0] for i in inv)) == wrap(sum(i[1] for i in inv)),
              "histo_weight_rel_err": abs(sum(i[2] for i in inv) - sum(i[3] for i in inv)) /
              max(1.0, sum(i[3] for i in inv))}

    # ---- the same windows through the operator interface: veneur_amd.Worker over the same D
    # engines (Worker.Flush hands the window's engine to its flush thread, as the reference's
    # Worker.Flush swaps the maps for the flusher, worker.go:276-284 / flusher.go:115-230; ingest
    # moves to the next engine at once).  One host thread drives it, as one Go worker would.
    worker_leg = None
    nw = args.steps if args.worker_windows < 0 else args.worker_windows
    if nw > 0 and not any(len(sl) for _, sl, _ in split_lists) and not sum(stream.split_counts):
        from veneur_amd.worker import Worker
        wk = Worker(engines=engines, percentiles=PCT)
        for _ in range(D):
            wk.process_batch(stream.batch)
            wk.flush_raw()
        wk.wait()
        sync()
        ctrl.barrier()
        tw = time.perf_counter()
        for _ in range(nw):
            wk.process_batch(stream.batch)
            fut = wk.flush_raw()
        wk.wait()
        sync()
        tw = time.perf_counter() - tw
        ctrl.barrier()
        tw = ctrl.max(tw)
        last = fut.result() if D > 1 else fut
        wk.close(close_engines=False)
        worker_leg = {"value": float(args.samples) * nw / tw, "unit": "samples/s", "ms_per_step": tw * 1e3 / nw,
                      "windows": nw, "engines": D,
                      "path": "veneur_amd.Worker(engines=D).process_batch(device batch) + flush_raw() per window: "
                              "Flush hands the window's engine to that engine's flush thread and returns, the "
                              "next window's ingest goes to the next engine (worker.go:276-284, "
                              "flusher.go:115-230); one host thread drives the worker",
                      "vs_harness": (float(args.samples) * nw / tw) / value}
        log(rank, "[bench] worker leg: %s" % json.dumps(worker_leg))

    # per-kernel timing (HIP events on the engine's stream) from extra, untimed steps: with
    # timing on, the phases run one after another so every launch is measured alone
    eng.timing_enable(True)
    tim = []
    for _ in range(args.timing_steps):
        last = step()
        tim.append(eng.timing())
    eng.timing_enable(False)
    if not tim:
        tim = [{k: 0.0 for k, _ in A.Timing._fields_}]
    for _ in range(args.profile_steps):
        last = step()
    mean = lambda k: float(np.mean([t[k] for t in tim]))
    kern = []
    for name, ms_k, by_k, n_k in (("k_histo_exact", "ms_histo_replay", "histo_replay_bytes", "histo_replay_launches"),
                                  ("k_set_segments", "ms_set_segments", "set_segment_bytes", "set_segment_launches"),
                                  ("k_radix_scatter", "ms_radix_scatter_total", "radix_scatter_bytes",
                                   "radix_scatter_launches"),
                                  ("k_part_scatter", "ms_part_scatter", "part_scatter_bytes", "part_scatter_launches")):
        ms, by, nl = mean(ms_k), mean(by_k), mean(n_k)
        if ms > 0 and nl > 0:
            ach = by / (ms * 1e-3) / 1e9
            kern.append({"kernel": name, "ms_per_step": ms, "launches_per_step": nl,
                         "algorithmic_bytes_per_launch": by / nl, "achieved": ach, "frac": ach / HBM_PEAK_GBS})
    # the counter aggregation (k_scalar_direct, one launch; 16 B per record of the window)
    ms_c = mean("ms_ingest_counter")
    if ms_c > 0:
        by_c = 16.0 * stream.counts[0]
        kern.append({"kernel": "counter aggregation", "ms_per_step": ms_c, "launches_per_step": 1.0,
                     "algorithmic_bytes_per_launch": by_c, "achieved": by_c / (ms_c * 1e-3) / 1e9,
                     "frac": by_c / (ms_c * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     # (tools/roofline_check.py: the trace's kernels of this phase, every launch summed)
                     "trace_kernels": ["k_part_count&CounterSrc", "k_part_scatter&CounterSrc", "k_counter_runs"],
                     "note": "the serialised counter phase: key-range partition pass (k_part_count, "
                             "k_part_scatter) + k_counter_runs (LDS sums per slot range, one device add per "
                             "touched slot per 128Ki-record slice)"})
    kern.sort(key=lambda k: -k["ms_per_step"])
    # the throughput view: each kernel class's algorithmic bytes per window over the window period
    # (ms_per_step, D windows in flight) -- what the class sustains in the pipelined headline,
    # against the latency view above (the class's own time in a serialised timing step)
    thr = [{"kernel": k["kernel"], "algorithmic_bytes_per_window": k["algorithmic_bytes_per_launch"] *
            k["launches_per_step"], "achieved": k["algorithmic_bytes_per_launch"] * k["launches_per_step"] /
            (ms_per_step * 1e-3) / 1e9} for k in kern]
    for t in thr:
        t["frac"] = t["achieved"] / HBM_PEAK_GBS
    phase = {k: round(mean(k), 4) for k in
             ("ms_ingest_counter", "ms_ingest_gauge", "ms_ingest_histo", "ms_ingest_set", "ms_flush")}
    top = kern[0] if kern else {}
    traffic, traffic_src, traffic_ratio = None, None, None
    tf = os.path.join(ROOT, "roofline_traffic.json")  # tools/pmc_traffic.py, PMC passes of this command
    if os.path.exists(tf) and top:
        with open(tf) as fh:
            tj = json.load(fh)
        if tj.get("kernel") == top["kernel"]:
            traffic_ratio = tj["traffic_over_algorithmic"]
            traffic, traffic_src = traffic_ratio * top["algorithmic_bytes_per_launch"], tj["source"]
    # whole path: SURVEY §8(d) algorithmic bytes of the window (16 B per scalar record, 8 B +
    # member bytes per set record, per-key state once) over the window's time
    n_sc = stream.counts[0] + stream.counts[1] + stream.counts[2] + stream.split_counts[0]
    n_set = stream.counts[3] + stream.split_counts[1]
    path_bytes = 16 * n_sc + 19 * n_set + 2 * (8 * n_slots[0] + 16 * n_slots[1] + 40 * n_slots[2])
    path_bytes = ctrl.sum(float(path_bytes))
    path_gbs = path_bytes / (ms_per_step * 1e-3) / 1e9 / world

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "window_latency_ms": window_latency_ms,
        "window_ingest_host_ms": window_ingest_ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64/u64",
        "data": "synthetic (one global DogStatsD-shaped C4 stream generated in HBM, seeded)",
        "config": {"workload": "C4 mixed counters/gauges/timers/sets, %d keys, %d samples per flush window over %d "
                               "GPU(s), Zipf(1.0), %s, %s" % (
                                   args.keys, args.samples, world,
                                   "hot keys split over the GPUs" if not args.no_split else "every key on its owner",
                                   "t-digest fast mode (geometric pieces past %d samples)" % args.exact_threshold
                                   if args.exact_threshold else "every t-digest merge replayed exactly"),
                   "histo_mode": "fast (non-conforming: rank-error bound 3e-3, not the reference's digests)"
                                 if args.exact_threshold else "exact",
                   "keys": args.keys, "samples_per_window": args.samples, "percentiles": list(PCT),
                   "compression": 100, "hll_precision": 14,
                   "parallelism": "key-sharded FNV %% %d + %d split hot keys (RCCL)" %
                                  (world, sum(len(split[c]) for c in split)),
                   "split_keys": {"counter": len(split[0]), "histo": len(split[2]), "set": len(split[3])},
                   "windows_in_flight": D,
                   "warmup_windows_run": warm,
                   "replay_reserved_cus": reserved,
                   "pipeline": ("%d engines per GPU take the windows in turn: window i + 1 is ingested while window "
                                "i's longest replays finish; every window ingested, replayed and flushed inside the "
                                "timed region (ms_per_step = timed region / steps; window_latency_ms = one window's "
                                "first call to its flush's return)" % D) if D > 1 else "one window at a time",
                   "split_key_choice": detect if detect is not None else
                   ("none" if args.no_split else "count of the stream's first 2^24 records (--sim-world)")},
        "roofline": {"bound": "hbm", "kernel": top.get("kernel"), "achieved": top.get("achieved"),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": top.get("frac"), "traffic": traffic,
                     "traffic_unit": "bytes per launch (HBM, PMC FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_over_algorithmic": traffic_ratio, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": top.get("algorithmic_bytes_per_launch"),
                     "launches_per_step": top.get("launches_per_step"), "ms_per_step": top.get("ms_per_step"),
                     "view": "latency: the kernel's algorithmic bytes over its own HIP-event time in a serialised "
                             "timing step (one engine, every launch measured alone, on the engine's stream)",
                     "kernels": kern},
        "roofline_throughput": {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "window_ms": ms_per_step,
                                "view": "throughput: each kernel class's algorithmic bytes per window over the "
                                        "pipelined window period ms_per_step (%d windows in flight)" % D,
                                "kernels": thr},
        "path": {"algorithmic_bytes_per_step": path_bytes, "effective_GBs_per_gpu": path_gbs,
                 "frac_of_hbm_peak": path_gbs / HBM_PEAK_GBS, "phase_ms_serialised_rank0": phase},
        "ranks": {"ms_per_step": rank_ms, "records": rank_records,
                  "imbalance_records_max_over_mean": max(rank_records) / (sum(rank_records) / len(rank_records)),
                  "imbalance_ms_max_over_mean": max(rank_ms) / (sum(rank_ms) / len(rank_ms))},
        "checks": checks,
    }
    if worker_leg is not None:
        result["worker_rotation"] = worker_leg

    # ---- PCIe-inclusive rate, CPU baseline and full-window parity (rank 0, N=1)
    if sim:
        result["simulated"] = "rank %d of %d on one GPU, no exchange partners: not a bench result" % (
            args.sim_rank, args.sim_world)
        dh = stream.to_host()
        hs = dh["h_slot"][:stream.counts[2]]
        result["sim"] = {"rank": args.sim_rank, "world": args.sim_world, "records": int(stream.n_records),
                         "largest_timer_key_samples": int(np.bincount(hs).max()) if len(hs) else 0}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not sim:
        t1 = time.time()
        d = stream.to_host()
        log(rank, "[bench] stream copied to the host in %.1fs" % (time.time() - t1))
        if args.pcie_steps > 0:
            hkw = dict(counters=(d["c_slot"][:stream.counts[0]], d["c_val"], d["c_rate"]),
                       gauges=(d["g_slot"], d["g_val"]),
                       histos=(d["h_slot"][:stream.counts[2]], d["h_val"][:stream.counts[2]],
                               d["h_rate"][:stream.counts[2]]),
                       sets=(d["s_slot"][:stream.counts[3]], d["s_off"][:stream.counts[3] + 1],
                             d["s_bytes"][:stream.counts[3] * 11]))

            def host_step():
                for c, slots, owners in split_lists:
                    if len(slots):
                        eng.split_keys(c, slots, owners)
                eng.ingest(**hkw)
                if sum(stream.split_counts):
                    eng.ingest_split_device(stream.split)
                return eng.flush_raw()
            host_step()
            sync()
            tp = time.perf_counter()
            for _ in range(args.pcie_steps):
                last = host_step()
            sync()
            pms = (time.perf_counter() - tp) * 1e3 / args.pcie_steps
            result["pcie_inclusive"] = {"value": args.samples / (pms * 1e-3), "unit": "samples/s", "ms_per_step": pms,
                                        "path": "vn_ingest_host from pageable host arrays (host checks + pinned "
                                                "staging + H2D + kernels); split-key records from HBM"}
        import oracle
        # num_workers = the CPUs this process may use: the GPU box's share is 16 of a machine whose
        # nproc counts every CPU of the host (the guide for the pool), so 16 unless fewer exist
        quota = cgroup_cpus()
        try:
            affinity = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            affinity = os.cpu_count() or 1
        # the CPUs this process may actually run on: the cgroup's CPU quota where one is set, the
        # affinity mask otherwise, and at most 16 (the GPU box's documented share per GPU)
        usable = min(affinity, quota) if quota else affinity
        threads = args.cpu_threads or max(1, min(16, usable))
        streams = {k: d[k] for k in ("c_slot", "c_val", "c_rate", "g_slot", "g_val", "h_slot", "h_val", "h_rate",
                                     "s_slot", "s_off", "s_bytes")}
        secs, _, ref = oracle.baseline_run_full(threads, n_slots, streams, PCT)
        model = "unknown"
        try:
            with open("/proc/cpuinfo") as fh:
                for line in fh:
                    if line.startswith("model name"):
                        model = line.split(":", 1)[1].strip()
                        break
        except OSError:
            pass
        result["cpu_baseline"] = {"value": args.samples / secs, "unit": "samples/s", "cores": threads,
                                  "kind": "port", "seconds": secs, "num_workers": threads,
                                  "nproc": os.cpu_count(), "cpus_affinity": affinity,
                                  "cgroup_cpu_quota": quota, "cpus_usable": usable, "cpu_model": model,
                                  "sample": "the full C4 flush window above (%d samples); C restatement of the Go "
                                            "Worker.ProcessMetric + flush path (oracle/), num_workers = %d worker "
                                            "threads routed by key digest %% num_workers (SURVEY 8(d)); usable CPUs "
                                            "= min(affinity %d, cgroup quota %s), capped at the box's share of 16"
                                            % (args.samples, threads, affinity, quota)}
        t1 = time.time()
        result["egress"] = egress_leg(last)
        log(rank, "[bench] egress leg in %.1fs: %s" % (time.time() - t1, json.dumps(result["egress"])))
        if args.text_lines > 0:
            t1 = time.time()
            result["text_intake"] = text_leg(args)
            log(rank, "[bench] text intake leg in %.1fs: %s" % (time.time() - t1, json.dumps(result["text_intake"])))
        o = last
        npct = len(PCT)
        arr = lambda p, n, dt: np.ctypeslib.as_array(p, shape=(n,)).copy() if n else np.zeros(0, dt)
        c_slot, c_val = arr(o.counter_slot, o.n_counter, np.uint32), arr(o.counter_value, o.n_counter, np.int64)
        g_slot, g_val = arr(o.gauge_slot, o.n_gauge, np.uint32), arr(o.gauge_value, o.n_gauge, np.float64)
        h_slot = arr(o.histo_slot, o.n_histo, np.uint32)
        h_q = arr(o.histo_quantiles, o.n_histo * npct, np.float64).reshape(-1, npct)
        h_st = arr(o.histo_stats, o.n_histo * 8, np.float64).reshape(-1, 8)
        s_slot, s_est = arr(o.set_slot, o.n_set, np.uint32), arr(o.set_estimate, o.n_set, np.uint64)
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
        # rank error: every key past the exact-replay threshold (split or hot remainder: the
        # approximated ones) plus a seeded sample of the others
        rng = np.random.default_rng(7)
        split_h = set((stream.split_slot0[2] + np.arange(len(split[2]))).tolist())
        cnt = np.bincount(d["h_slot"], minlength=n_slots[2])
        # (the exact mode approximates nothing; its keys past 32768 samples -- the ones the fast
        # mode would take through geometric pieces -- are all checked)
        big = set(np.nonzero(cnt > (args.exact_threshold or 32768))[0].tolist())
        pick = np.array(sorted(split_h | big | set(rng.choice(h_slot, min(args.parity_keys, len(h_slot)),
                                                              replace=False).tolist())), np.uint32)
        idx = np.searchsorted(h_slot, pick)
        errs, acc_e, acc_r = rank_error_stats(d, pick, h_q[idx], ref["histo_q"][pick])
        par["rank_error_keys"] = int(len(pick))
        par["rank_error_max"] = {("p%g" % (100 * p)): float(errs[:, k].max()) for k, p in enumerate(PCT)}
        par["rank_error_mean"] = {("p%g" % (100 * p)): float(errs[:, k].mean()) for k, p in enumerate(PCT)}
        for name, sel in (("split", split_h), ("past_exact_threshold", big)):
            m = np.isin(pick, list(sel))
            if m.any():
                par["rank_error_max_%s_keys" % name] = {("p%g" % (100 * p)): float(errs[m, k].max())
                                                        for k, p in enumerate(PCT)}
                par["%s_keys" % name] = int(m.sum())
        # keys past the threshold: how far each side is from the key's exact quantile, |F(q) - p|
        # (the reference's sequential 42-sample merge is itself an approximation); and for the
        # keys whose rank error passes 1e-3, which side is nearer the exact quantile
        mb = np.isin(pick, list(big))
        if mb.any():
            pk = lambda a, f: {("p%g" % (100 * p)): float(f(a[mb, k])) for k, p in enumerate(PCT)}
            over = errs[mb] > 1e-3
            par["accuracy_vs_exact_quantile_past_threshold"] = {
                "engine_max": pk(acc_e, np.max), "reference_max": pk(acc_r, np.max),
                "engine_mean": pk(acc_e, np.mean), "reference_mean": pk(acc_r, np.mean),
                "quantiles_with_rank_error_over_1e-3": int(over.sum()),
                "of_those_engine_nearer_exact": int((acc_e[mb][over] < acc_r[mb][over]).sum())}
        worst = np.argsort(-errs.max(axis=1))[:8]
        par["rank_error_worst_keys"] = [{"slot": int(pick[i]), "samples": int(cnt[pick[i]]),
                                         "split": int(pick[i]) in split_h,
                                         "err": [round(float(x), 7) for x in errs[i]],
                                         "engine_vs_exact": [round(float(x), 7) for x in acc_e[i]],
                                         "reference_vs_exact": [round(float(x), 7) for x in acc_r[i]]}
                                        for i in worst]
        par["quantiles_bit_exact_frac"] = float(np.mean(np.all(h_q == ref["histo_q"][h_slot], axis=1)))
        result["p99_rank_error"] = par["rank_error_max"]["p99"]
        result["parity"] = par
        log(rank, "[bench] parity checked in %.1fs" % (time.time() - t1))
    if args.c5_hosts > 0 and not sim:
        # C5 on every rank: each keeps the imports of the keys it owns (no collective)
        t1 = time.time()
        c5 = c5_leg(args, rank, world, ctrl, local_rank)
        if rank == 0:
            result["c5"] = c5
            log(rank, "[bench] C5 leg in %.1fs: %s" % (time.time() - t1, json.dumps(c5)))
    if rank == 0:
        if exact_prof is not None:
            result["exact_prof_block0"] = exact_prof
        print(json.dumps(result), flush=True)
    for e in engines:
        e.close()
    stream.free()
    if comm is not None:
        comm.close()
    ctrl.close()


if __name__ == "__main__":
    main()
