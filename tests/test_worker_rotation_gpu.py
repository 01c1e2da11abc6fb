"""Worker.Flush with D engines taking the windows in turn (veneur_amd.Worker(pipeline=D)), on the GPU.

The reference's Worker.Flush swaps in fresh maps and returns; the flusher works on the swapped
ones while the worker takes the next interval (worker.go:276-284, flusher.go:115-230).  The Worker
does the same with D engines: each window is ingested into one engine, whose flush then runs on a
thread of its own while the next window goes to the next engine.  Every window must equal the
restated Go worker fed that window alone: counters, gauges and set estimates bit-exact, histogram
weight / min / max exact and every quantile bit-identical.
"""
import numpy as np
import pytest

import veneur_amd as V
from tests.util import PCT, run_oracle
from veneur_amd import worker as W

pytestmark = pytest.mark.gpu


def _windows(n, n_keys, n_samples):
    return [V.synth(seed=9100 + i, n_keys=n_keys, n_samples=n_samples, member_universe=2_000_000) for i in range(n)]


def _check(f, d):
    n = d["n_slots"]
    w = run_oracle(d, n)
    assert dict(zip(f.counter_slot.tolist(), f.counter_value.tolist())) == \
        {s: w.counter_value(s) for s in range(n[0]) if w.touched(0, s)}
    assert dict(zip(f.gauge_slot.tolist(), f.gauge_value.tolist())) == \
        {s: w.gauge_value(s) for s in range(n[1]) if w.touched(1, s)}
    assert dict(zip(f.set_slot.tolist(), f.set_estimate.tolist())) == \
        {s: w.set_estimate(s) for s in range(n[3]) if w.touched(3, s)}
    ost = np.array([w.histo_stats(int(s)) for s in f.histo_slot])
    assert np.array_equal(f.histo_stats[:, :3], ost[:, :3])
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    assert np.array_equal(f.histo_quantiles, oq)
    return int(np.bincount(d["h_slot"]).max()) if len(d["h_slot"]) else 0


def test_worker_three_engines_seven_windows_match_oracle_per_window():
    """D = 3 engines over 7 windows of 2M samples (the longest timer keys take the long-key
    replays; the batched one, from 524288 samples, is covered by test_batch_replay_gpu.py): each
    window's flush equals the oracle of that window alone."""
    ws = _windows(7, 2000, 2_000_000)
    cap = tuple(max(max(d["n_slots"][c] for d in ws), 1) for c in range(4))
    nrec = max(max(len(d["c_slot"]), len(d["g_slot"]), len(d["h_slot"]), len(d["s_slot"])) for d in ws) + 1
    w = W.Worker(capacity=cap, percentiles=PCT, batch_records=nrec, pipeline=3)
    assert w.pipeline == 3 and w.percentiles == PCT
    futs, longest = [], 0
    try:
        for d in ws:
            w.process_batch(counters=(d["c_slot"], d["c_val"], d["c_rate"]), gauges=(d["g_slot"], d["g_val"]),
                            histos=(d["h_slot"], d["h_val"], d["h_rate"]),
                            sets=(d["s_slot"], d["s_off"], d["s_bytes"]))
            futs.append(w.flush_raw(copy=True))
        for f, d in zip(futs, ws):
            out = f.result(timeout=120)
            assert out.samples_processed == sum(len(d[k]) for k in ("c_slot", "g_slot", "h_slot", "s_slot"))
            longest = max(longest, _check(out, d))
    finally:
        w.close()
    assert longest >= 20000  # keys of tens of thousands of samples in at least one window


def test_worker_in_turn_maps_equal_single_engine():
    """The same ProcessMetric / ImportMetric / Flush sequence through Worker(pipeline=3) and
    Worker(pipeline=1): identical WorkerMetrics window by window (InterMetrics compared by name,
    tags and value bits)."""
    rng = np.random.default_rng(5)
    windows = []
    for i in range(6):
        ms = []
        for j in range(3000):
            k = int(rng.integers(0, 40))
            t = ("counter", "gauge", "timer", "set", "histogram")[k % 5]
            v = ("m%d" % rng.integers(0, 500)) if t == "set" else float(np.round(rng.lognormal(2, 1), 3))
            ms.append(W.UDPMetric(W.MetricKey("k%d" % k, t, "env:%d" % (k % 3)), v,
                                  sample_rate=(0.5 if j % 7 == 0 else 1.0), tags=["env:%d" % (k % 3)]))
        windows.append(ms)
    res = []
    for D in (1, 3):
        w = W.Worker(capacity=(64, 64, 64, 64), percentiles=PCT, batch_records=1 << 10, pipeline=D)
        try:
            wms = []
            for ms in windows:
                for m in ms:
                    w.ProcessMetric(m)
                wms.append(w.Flush())
            res.append([sorted((m.name, tuple(m.tags), np.float64(m.value).tobytes())
                               for m in W.generate_inter_metrics([wm], list(PCT), list(PCT), W.DEFAULT_AGGREGATES,
                                                                 False))
                        for wm in wms])
        finally:
            w.close()
    assert res[0] == res[1]


def test_worker_in_turn_flush_datadog_shared_sink_equals_single_engine():
    """One DatadogSink serving D = 3 engines' flush threads (their flushes overlap, each calls
    vn_datadog_flush on the same vn_sink): every window's bodies equal those of D = 1."""
    from veneur_amd.sink import DatadogSink
    rng = np.random.default_rng(11)
    windows = []
    for i in range(8):
        ms = []
        for j in range(4000):
            k = int(rng.integers(0, 300))
            t = ("counter", "gauge", "timer", "set", "histogram")[k % 5]
            v = ("m%d" % rng.integers(0, 900)) if t == "set" else float(np.round(rng.lognormal(2, 1), 3))
            ms.append(W.UDPMetric(W.MetricKey("k%d" % k, t, "env:%d" % (k % 3)), v, tags=["env:%d" % (k % 3)]))
        windows.append(ms)
    agg = W.HistogramAggregates(W.Aggregate.AggregateMin | W.Aggregate.AggregateMax | W.Aggregate.AggregateCount |
                                W.Aggregate.AggregateMedian)
    res = []
    for D in (1, 3):
        w = W.Worker(capacity=(512,) * 4, percentiles=PCT, batch_records=1 << 10, pipeline=D)
        sink = DatadogSink(10.0, "h", ["dc:1"], 50)
        try:
            outs = []
            for ms in windows:
                for m in ms:
                    w.ProcessMetric(m)
                outs.append(w.flush_datadog(sink, (0.9, 0.99), agg, timestamp=1234))
            res.append([o.result(timeout=120) if D > 1 else o for o in outs])
        finally:
            w.close()
            sink.close()
    assert res[0] == res[1]
    assert all(r[1][0] > 0 for r in res[0])
