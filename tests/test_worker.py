"""veneur_amd.Worker: veneur's Worker / samplers API over the HIP engine.

The CPU tests check the host logic with a recording stand-in engine (scope routing of Upsert,
staging order around imports, the panics and logged errors, Histo.Flush's InterMetrics); the
GPU tests run the reference's worker_test.go / samplers_test.go cases through the real engine
and compare a random DogStatsD-shaped stream's InterMetrics with the restated Go worker.
"""
import math
import struct

import numpy as np
import pytest

import oracle
from veneur_amd import worker as W
from veneur_amd.engine import EngineError, FlushOutput

K = W.MetricKey


def go_i64(x):
    """Go's float64 -> int64 conversion on amd64 (CVTTSD2SQ): NaN and out-of-range give MinInt64."""
    if x != x or not (-9.223372036854775808e18 < x < 9.223372036854775808e18):
        return -(1 << 63)
    return int(x)


class RecordingEngine:
    """Stands in for veneur_amd.Engine: records the calls, flushes counters as sums."""

    def __init__(self, capacity=(8, 8, 8, 8), percentiles=(0.5, 0.9)):
        self.capacity, self.percentiles, self.calls = capacity, percentiles, []
        self.cval = {}
        self.hvals = {}

    def ingest(self, **kw):
        self.calls.append(("ingest", {k: [a.tolist() for a in v] for k, v in kw.items()}))
        if "histos" in kw:
            for s, v, r in zip(*kw["histos"]):
                self.hvals.setdefault(int(s), []).append(float(v))
        if "counters" in kw:
            for s, v, r in zip(*kw["counters"]):
                with np.errstate(divide="ignore", invalid="ignore"):
                    inv = float(np.float32(1) / np.float32(r))
                x = self.cval.get(int(s), 0) + go_i64(float(v)) * go_i64(inv)
                self.cval[int(s)] = (x + (1 << 63)) % (1 << 64) - (1 << 63)  # wrapping int64

    def import_counters(self, slot, v):
        self.calls.append(("import_counters", slot.tolist(), v.tolist()))
        for s_, x in zip(slot.tolist(), v.tolist()):
            self.cval[int(s_)] = self.cval.get(int(s_), 0) + int(x)

    def import_gauges(self, slot, v):
        self.calls.append(("import_gauges", slot.tolist(), v.tolist()))

    def import_histos(self, slot, p):
        if any(x == b"bad" for x in p):  # the engine applies nothing of a failing batch
            raise EngineError("malformed (rc=-4)")
        self.calls.append(("import_histos", slot.tolist()))

    def import_sets(self, slot, p):
        self.calls.append(("import_sets", slot.tolist()))

    def export_histos(self, slots):
        return [b"gob%d" % s for s in slots]

    def export_sets(self, slots):
        return [b"hll%d" % s for s in slots]

    def flush(self, histo_quantile_mask=None, set_estimate_mask=None):
        self.calls.append(("flush",))
        self.masks = (histo_quantile_mask, set_estimate_mask)
        cs = sorted(self.cval)
        hs = sorted(self.hvals)
        z = np.zeros(0, np.uint32)
        hst = np.array([[len(v), min(v), max(v), sum(v), sum(1 / x for x in v), min(v), max(v), len(v)]
                        for v in (self.hvals[s] for s in hs)]).reshape(-1, 8)
        out = FlushOutput(np.array(cs, np.uint32), np.array([self.cval[s] for s in cs], np.int64), z, np.zeros(0),
                          np.array(hs, np.uint32), hst, np.full((len(hs), len(self.percentiles)), 1.0), z,
                          np.zeros(0, np.uint64), np.zeros(0, np.uint8), 0, 0)
        self.cval = {}
        self.hvals = {}
        return out


def cpu_worker(**kw):
    return W.Worker(engine=RecordingEngine(**kw), batch_records=1000)


def test_worker_counter_flush_and_empty_window():  # worker_test.go:11-30
    w = cpu_worker()
    w.ProcessMetric(W.UDPMetric(K("a.b.c", "counter"), 1.0, 1.0, digest=12345))
    wm = w.Flush()
    assert len(wm.counters) == 1 and wm.counters[K("a.b.c", "counter")].value == 1
    assert len(w.Flush().counters) == 0


def test_worker_local_and_global_maps():  # worker_test.go:32-83
    w = cpu_worker()
    w.ProcessMetric(W.UDPMetric(K("a.b.c", "histogram"), 1.0, scope=W.MetricScope.LocalOnly))
    w.ProcessMetric(W.UDPMetric(K("a.b.c", "counter"), 1.0, scope=W.MetricScope.GlobalOnly))
    w.ProcessMetric(W.UDPMetric(K("b.c.a", "gauge"), 1.0, scope=W.MetricScope.GlobalOnly))
    w.ProcessMetric(W.UDPMetric(K("t", "timer"), 2.0, scope=W.MetricScope.LocalOnly))
    w.ProcessMetric(W.UDPMetric(K("s", "set"), "x", scope=W.MetricScope.LocalOnly))
    wm = w.Flush()
    assert (len(wm.local_histograms), len(wm.histograms)) == (1, 0)
    assert (len(wm.global_gauges), len(wm.gauges)) == (1, 0)
    assert (len(wm.global_counters), len(wm.counters)) == (1, 0)
    assert (len(wm.local_timers), len(wm.local_sets)) == (1, 1)


def test_worker_same_key_different_maps_get_different_slots():
    w = cpu_worker()
    w.ProcessMetric(W.UDPMetric(K("a", "counter"), 3.0))
    w.ProcessMetric(W.UDPMetric(K("a", "counter"), 4.0, scope=W.MetricScope.GlobalOnly))
    w.ProcessMetric(W.UDPMetric(K("a", "counter"), 5.0, 0.5))
    wm = w.Flush()
    assert wm.counters[K("a", "counter")].value == 13 and wm.global_counters[K("a", "counter")].value == 4


def test_worker_import_drains_staged_samples_first():  # arrival order across ProcessMetric / ImportMetric
    w = cpu_worker()
    w.ProcessMetric(W.UDPMetric(K("g", "gauge"), 1.0, scope=W.MetricScope.GlobalOnly))
    w.ImportMetric(W.JSONMetric(K("g", "gauge"), [], struct.pack("<d", 7.0)))
    w.ImportMetric(W.JSONMetric(K("c", "counter"), [], struct.pack("<q", 9)))
    names = [c[0] for c in w.engine.calls]
    assert names == ["ingest", "import_gauges", "import_counters"]
    assert w.engine.calls[1][1:] == ([0], [7.0])
    assert w.imported == 2 and w.processed == 1
    wm = w.Flush()
    assert wm.global_counters[K("c", "counter")].value == 9 and len(wm.global_gauges) == 1


def test_worker_errors_like_the_reference(caplog):
    w = cpu_worker()
    with pytest.raises(ValueError, match="invalid value added"):  # merging_digest.go:98-100 panic
        w.ProcessMetric(W.UDPMetric(K("h", "histogram"), float("nan")))
    w.ProcessMetric(W.UDPMetric(K("x", "distribution"), 1.0))  # logged, counted
    w.ImportMetric(W.JSONMetric(K("h", "histogram"), [], b"bad"))  # Combine error: logged, skipped
    w.ImportMetric(W.JSONMetric(K("c", "counter"), [], b"\x01"))
    assert "Unknown metric type" in caplog.text and "Could not merge" in caplog.text
    assert w.processed == 2 and w.imported == 2
    with pytest.raises(OverflowError):
        for i in range(20):
            w.ProcessMetric(W.UDPMetric(K("k%d" % i, "counter"), 1.0))


def _histo_view(vals, tags=("a:b",)):
    """The Histo a window of samples flushes to (statistics from the restated Go sampler)."""
    w = oracle.Worker(1, 1, 1, 1)
    w.histo(np.zeros(len(vals), np.uint32), np.array(vals, float), np.ones(len(vals), np.float32))
    st = w.histo_stats(0)
    q = {p: w.histo_quantile(0, p) for p in (0.5, 0.9, 0.99, 0.999)}
    return W.Histo("a.b.c", list(tags), st[0], st[1], st[2], st[3], st[4], q)


def test_histo_flush_intermetrics():  # samplers_test.go:192-283
    h = _histo_view([5, 10, 15, 20, 25])
    A = W.Aggregate
    agg = W.HistogramAggregates(A.AggregateMin | A.AggregateMax | A.AggregateMedian | A.AggregateAverage |
                                A.AggregateCount | A.AggregateSum | A.AggregateHarmonicMean, 7)
    m = h.flush(10, [0.90], agg)
    assert len(m) == agg.count + 1
    assert [x.name for x in m] == ["a.b.c.max", "a.b.c.min", "a.b.c.sum", "a.b.c.avg", "a.b.c.count",
                                   "a.b.c.median", "a.b.c.hmean", "a.b.c.90percentile"]
    assert [x.value for x in m[:6]] == [25, 5, 75, 15, 5, 15]
    assert m[6].value == 5 / (1 / 5 + 1 / 10 + 1 / 15 + 1 / 20 + 1 / 25)
    assert m[7].value == 23.75
    assert m[4].type == W.MetricType.CounterMetric and all(x.type == W.MetricType.GaugeMetric for x in m if
                                                           x.name != "a.b.c.count")
    assert all(x.tags == ["a:b"] for x in m)


def test_histo_flush_single_aggregates_and_guards():  # samplers_test.go:285-352; samplers.go:380-452 guards
    h = _histo_view([5, 10, 15, 20, 25])
    assert [(x.name, x.value) for x in h.flush(10, [], W.HistogramAggregates(W.Aggregate.AggregateAverage, 1))] == \
        [("a.b.c.avg", 15.0)]
    hm = h.flush(10, [], W.HistogramAggregates(W.Aggregate.AggregateHarmonicMean, 1))
    assert len(hm) == 1 and hm[0].name == "a.b.c.hmean"
    empty = W.Histo("e", [], 0.0, math.inf, -math.inf, 0.0, 0.0, {0.5: float("nan")})
    assert [x.name for x in empty.flush(10, [], W.DEFAULT_AGGREGATES)] == []
    assert h.flush(10, [0.999], W.HistogramAggregates())[0].name == "a.b.c.99percentile"  # Go's int(p*100)
    with pytest.raises(ValueError):
        h.flush(10, [0.75], W.HistogramAggregates())


def test_route_info_and_exports():  # samplers.go:104-122, 150-234
    assert W.route_info(["a:b", "veneursinkonly:datadog", "veneursinkonly:kafka"]) == {"datadog", "kafka"}
    assert W.route_info(["a:b"]) is None
    c = W.Counter("c", ["x:y"], -5)
    assert c.export().value == struct.pack("<q", -5) and c.flush(10)[0].type == W.MetricType.CounterMetric
    g = W.Gauge("g", [], 2.5)
    assert g.export().value == struct.pack("<d", 2.5)
    with pytest.raises(ValueError):
        W.Set("s", [], 3, True).export()


def test_import_routing_kats():  # http_test.go:23-57
    ms = [W.JSONMetric(K(n, t), [], b"") for n, t in (("foo", "histogram"), ("bar", "set"), ("baz", "counter"),
                                                      ("qux", "gauge"))]
    assert [W.metric_digest(m.key) % 96 for m in ms] == [0x4F, 0x3A, 0x2, 0x3C]
    chunks = list(W.json_metrics_by_worker(ms, 96))
    assert [(c[0].key.name, w) for c, w in chunks] == [("baz", 2), ("bar", 0x3A), ("qux", 0x3C), ("foo", 0x4F)]
    # the import hash equals the parser's digest of "foo:1|h|#bar" (restated in the oracle)
    assert W.metric_digest(K("foo", "histogram", "bar")) == oracle.metric_digest("foo", "histogram", "bar")


def test_import_metrics_and_udp_routing_reach_the_right_workers():
    ws = [cpu_worker() for _ in range(3)]
    ms = [W.JSONMetric(K("c%d" % i, "counter"), [], struct.pack("<q", i)) for i in range(12)]
    W.import_metrics(ws, ms)
    for w in ws:
        got = w.Flush().global_counters
        assert all(W.metric_digest(k) % 3 == ws.index(w) for k in got)
        assert all(got[k].value == int(k.name[1:]) for k in got)
    u = W.UDPMetric(K("x", "counter"), 2.0)
    W.route_udp(ws, u)
    assert len(ws[W.metric_digest(u.key) % 3].Flush().counters) == 1


# ------------------------------------------------------------------ through the engine (GPU)
def gpu_worker(**kw):
    return W.Worker(capacity=(64, 64, 64, 64), percentiles=(0.5, 0.9, 0.99), batch_records=4096, **kw)


@pytest.mark.gpu
def test_gpu_worker_reference_cases():  # worker_test.go:11-117, samplers_test.go:73-80, 144-168, 192-283
    w = gpu_worker()
    try:
        w.ProcessMetric(W.UDPMetric(K("a.b.c", "counter"), 1.0, 1.0, digest=12345))
        w.ProcessMetric(W.UDPMetric(K("rate", "counter"), 5.0, 0.5))
        for v in (5, 10, 15, 20, 25):
            w.ProcessMetric(W.UDPMetric(K("a.b.c", "histogram", "a:b"), float(v), tags=["a:b"]))
        for m in ("5", "5", "123", "2147483647", "-2147483648"):
            w.ProcessMetric(W.UDPMetric(K("s", "set", "a:b"), m, tags=["a:b"]))
        # a forwarded set and histogram (Set.Export / Histo.Export of local samplers)
        sk = oracle.Sketch()
        sk.insert(b"foo"), sk.insert(b"bar")
        w.ImportMetric(W.JSONMetric(K("imp", "set"), [], sk.marshal()))
        td = oracle.MergingDigest(100.0)
        td.add(1.0), td.add(2.0)
        w.ImportMetric(W.JSONMetric(K("imp", "histogram"), [], td.gob_encode()))
        wm = w.Flush()
        assert wm.counters[K("a.b.c", "counter")].value == 1 and wm.counters[K("rate", "counter")].value == 10
        h = wm.histograms[K("a.b.c", "histogram", "a:b")]
        A = W.Aggregate
        m = h.flush(10, [0.9], W.HistogramAggregates(A.AggregateMin | A.AggregateMax | A.AggregateMedian |
                                                      A.AggregateAverage | A.AggregateCount | A.AggregateSum |
                                                      A.AggregateHarmonicMean, 7))
        assert [x.value for x in m[:6]] + [m[7].value] == [25, 5, 75, 15, 5, 15, 23.75]
        assert wm.sets[K("s", "set", "a:b")].flush()[0].value == 4
        assert len(wm.sets) == 2 and len(wm.histograms) == 2
        assert wm.sets[K("imp", "set")].estimate == 2
        assert wm.histograms[K("imp", "histogram")].quantile(0.5) == td.quantile(0.5)
        assert len(w.Flush()) == 0
    finally:
        w.close()


@pytest.mark.gpu
def test_gpu_worker_random_stream_matches_restated_go():
    rng = np.random.default_rng(7)
    keys = [K("m%d" % i, t, "env:%d" % (i % 3)) for i, t in
            enumerate(["counter", "gauge", "histogram", "timer", "set"] * 8)]
    scopes = [W.MetricScope(int(x)) for x in rng.integers(0, 3, len(keys))]
    w = gpu_worker()
    o = oracle.Worker(64, 64, 64, 64)
    slots, nxt = {}, [0, 0, 0, 0]
    cls_of = {"counter": 0, "gauge": 1, "histogram": 2, "timer": 2, "set": 3}
    try:
        for _ in range(3000):
            i = int(rng.integers(0, len(keys)))
            k, sc = keys[i], scopes[i]
            rate = float(rng.choice([1.0, 0.5, 0.1]))
            v = ("u%d" % rng.integers(0, 500)) if k.type == "set" else float(np.round(rng.lognormal(3, 1), 3))
            w.ProcessMetric(W.UDPMetric(k, v, rate, tags=[k.joined_tags], scope=sc))
            mp = W._map_for(k.type, sc)
            cls = cls_of[k.type]
            if (mp, k) not in slots:  # slots are dense per class in order of first Upsert
                slots[(mp, k)] = nxt[cls]
                nxt[cls] += 1
            s = slots[(mp, k)]
            feed(o, cls, s, v, rate)
        wm = w.Flush(forward=True)
        for k, sc in zip(keys, scopes):
            mp = W._map_for(k.type, sc)
            smp = getattr(wm, mp)[k]
            s = slots[(mp, k)]
            cls = cls_of[k.type]
            if cls == 0:
                assert smp.value == o.counter_value(s)
            elif cls == 1:
                assert smp.value == o.gauge_value(s)
            elif cls == 2:
                st = o.histo_stats(s)
                assert (smp.local_weight, smp.local_min, smp.local_max) == tuple(st[:3])
                assert smp.quantile(0.99) == o.histo_quantile(s, 0.99)  # few samples: exact replay
                if mp in ("histograms", "timers"):
                    assert smp.export().value == o.histo_gob(s)
            else:  # Set.Export before Estimate: the restated Estimate merges the tmpSet (hyperloglog.go:204)
                if mp == "sets":
                    assert smp.export().value == o.set_sketch(s).marshal()
                assert smp.estimate == o.set_estimate(s)
    finally:
        w.close()


def feed(o, cls, s, v, rate):
    one = np.array([s], np.uint32)
    if cls == 0:
        o.counter(one, np.array([v]), np.array([rate], np.float32))
    elif cls == 1:
        o.gauge(one, np.array([v]))
    elif cls == 2:
        o.histo(one, np.array([v]), np.array([rate], np.float32))
    else:
        b = v.encode()
        o.set(one, np.array([0, len(b)], np.uint32), np.frombuffer(b, np.uint8))


def _names(ims):
    return sorted(m.name for m in ims)


def test_generate_inter_metrics_local_and_global_rules():
    """generateInterMetrics (flusher.go:168-230): a local veneur flushes no percentiles of mixed
    histograms/timers, no mixed sets, global counters or global gauges -- those are forwarded --
    while local-only histograms keep their percentiles; a global veneur flushes everything."""
    def feed(w):
        for v in (1.0, 2.0, 7.0, 8.0, 100.0):
            w.ProcessMetric(W.UDPMetric(K("a.b.c", "histogram"), v))                              # mixed
            w.ProcessMetric(W.UDPMetric(K("l.h", "histogram"), v, scope=W.MetricScope.LocalOnly))
            w.ProcessMetric(W.UDPMetric(K("t.m", "timer"), v))
        for _ in range(40):
            w.ProcessMetric(W.UDPMetric(K("x.y.z", "counter"), 1.0, scope=W.MetricScope.LocalOnly))
        w.ProcessMetric(W.UDPMetric(K("g.c", "counter"), 3.0, scope=W.MetricScope.GlobalOnly))
        w.ProcessMetric(W.UDPMetric(K("g.g", "gauge"), 3.0, scope=W.MetricScope.GlobalOnly))
        w.ProcessMetric(W.UDPMetric(K("s", "set"), "a"))
        w.ProcessMetric(W.UDPMetric(K("ls", "set"), "a", scope=W.MetricScope.LocalOnly))

    pct = (0.5, 0.75, 0.99)
    w = W.Worker(engine=RecordingEngine(percentiles=pct), batch_records=1000, percentiles=pct)
    feed(w)
    final, fwd = W.server_flush([w], True, pct)
    assert _names(final) == sorted(["x.y.z", "a.b.c.max", "a.b.c.min", "a.b.c.count", "t.m.max", "t.m.min",
                                    "t.m.count", "l.h.max", "l.h.min", "l.h.count", "l.h.50percentile",
                                    "l.h.75percentile", "l.h.99percentile", "ls"])
    assert sorted((m.key.name, m.key.type) for m in fwd) == [("a.b.c", "histogram"), ("g.c", "counter"),
                                                              ("g.g", "gauge"), ("s", "set"), ("t.m", "timer")]
    qmask, emask = w.engine.masks
    win_slots = {"a.b.c": 0, "l.h": 1, "t.m": 2}  # histo slots in upsert order
    assert qmask[win_slots["l.h"]] == 1 and qmask[win_slots["a.b.c"]] == 0 and qmask[win_slots["t.m"]] == 0
    assert emask[0] == 0 and emask[1] == 1  # sets: "s" (mixed) then "ls" (local-only)

    g = W.Worker(engine=RecordingEngine(percentiles=pct), batch_records=1000, percentiles=pct)
    feed(g)
    final, fwd = W.server_flush([g], False, pct)
    assert fwd == [] and g.engine.masks == (None, None)
    names = _names(final)
    for n in ("a.b.c.50percentile", "t.m.99percentile", "s", "g.c", "g.g", "ls", "l.h.75percentile"):
        assert n in names


def test_nan_sample_rate_counter_sampled_histogram_dropped():
    """A NaN rate passes the parser (parser.go:262-272, both comparisons false).  A counter samples
    it as Go does: int64(sample) * int64(float32(1/NaN)) = sample * MinInt64, wrapping
    (samplers.go:133) -- 2 * MinInt64 wraps to 0, 3 * MinInt64 to MinInt64.  A histogram's NaN
    weight would never finish Go's next merge (test_oracle_kats.py::test_nan_weight_merge_never_ends):
    the Worker drops that one record and keeps the rest of the staged batch."""
    from veneur_amd import parser as P
    w = W.Worker(engine=RecordingEngine(capacity=(8, 8, 8, 8)), batch_records=4)
    lines = [b"a:1|c", b"a:2|c|@nan", b"b:5|h|@nan", b"a:3|c", b"a:4|c", b"a:5|c", b"c:3|c|@nan"]
    for ln in lines:
        m = P.parse_metric(ln)
        w.ProcessMetric(m)
    assert w.dropped == 1
    wm = w.Flush()
    assert wm.counters[K("a", "counter")].value == 1 + 3 + 4 + 5
    assert wm.counters[K("c", "counter")].value == -(1 << 63)
    assert K("b", "histogram") not in wm.histograms


def test_non_utf8_set_member_and_name_bytes():
    """Invalid UTF-8 in a set member or name reaches the engine as the raw bytes (Go inserts the
    bytes into the HLL and hashes them into the digest)."""
    from veneur_amd import parser as P
    w = W.Worker(engine=RecordingEngine(), batch_records=1000)
    m = P.parse_metric(b"s\xfe:\xff\x80|s")
    w.ProcessMetric(m)
    assert W.metric_digest(m.key) == oracle.fnv1a32(b"s\xfe", b"set", b"")
    w._drain()
    call = [c for c in w.engine.calls if c[0] == "ingest"][-1][1]
    assert bytes(call["sets"][2]) == b"\xff\x80"


def test_set_member_bytes_drain_before_engine_limit():
    """Long members: the staged member bytes never pass the engine's max_batch_member_bytes."""
    eng = RecordingEngine()
    eng.max_batch_member_bytes = 1000
    w = W.Worker(engine=eng, batch_records=10000)
    for i in range(200):
        w.ProcessMetric(W.UDPMetric(K("s", "set"), ("%03d" % i) * 30))  # 90-byte members
    w.Flush()
    sizes = [len(c[1]["sets"][2]) for c in eng.calls if c[0] == "ingest" and "sets" in c[1]]
    assert sum(sizes) == 200 * 90 and max(sizes) <= 1000


def test_import_lone_surrogate_name_is_replaced():
    """encoding/json decodes an escaped lone surrogate as U+FFFD (the digest must not crash)."""
    from veneur_amd import http_import as H
    body = b'[{"name":"a\\ud800b","type":"counter","tagstring":"","tags":null,"value":"AQAAAAAAAAA="}]'
    ms = H.unmarshal_metrics_from_http(body, "")
    assert ms[0].key.name == "a\ufffdb"
    W.metric_digest(ms[0].key)


@pytest.mark.gpu
def test_gpu_local_and_global_server_flush():
    """server_test.go TestLocalServerMixedMetrics (303-416), TestLocalServerUnaggregatedMetrics
    (239-270) and TestGlobalServerFlush (272-301) through the engine: percentiles [.5 .75 .99],
    aggregates min/max/count."""
    from veneur_amd import http_import as H
    pct = (0.5, 0.75, 0.99)
    vals = (1.0, 2.0, 7.0, 8.0, 100.0)
    # local veneur: mixed histogram forwarded (no percentiles on the engine), local counter flushed
    w = W.Worker(capacity=(64, 64, 64, 64), percentiles=pct, batch_records=4096)
    try:
        for v in vals:
            w.ProcessMetric(W.UDPMetric(K("a.b.c", "histogram"), v, 1.0, digest=12345))
        for _ in range(40):
            w.ProcessMetric(W.UDPMetric(K("x.y.z", "counter"), 1.0, 1.0, digest=12345, scope=W.MetricScope.LocalOnly))
        w.ProcessMetric(W.UDPMetric(K("s", "set"), "m"))
        final, fwd = W.server_flush([w], True, pct)
        byname = {m.name: m.value for m in final}
        assert byname == {"x.y.z": 40.0, "a.b.c.max": 100.0, "a.b.c.min": 1.0, "a.b.c.count": 5.0}
        assert [(m.key.name, m.key.type) for m in fwd] == [("a.b.c", "histogram"), ("s", "set")]
        # the global receives the histogram's digest: centroids {1,2,7,8,100}, min 1, max 100
        exp = oracle.MergingDigest(100.0)
        with open("tests/golden/tdigest_1_2_7_8_100.gob", "rb") as fh:
            exp.gob_decode(fh.read())
        got = oracle.MergingDigest(100.0)
        got.gob_decode(fwd[0].value)
        for a, b in zip(got.centroids(), exp.centroids()):
            np.testing.assert_array_equal(a, b)
        assert (got.min(), got.max(), got.count()) == (1.0, 100.0, 5.0)
        # the global veneur: import the forward, flush everything
        g = W.Worker(capacity=(64, 64, 64, 64), percentiles=pct, batch_records=4096)
        try:
            H.import_metrics([g], fwd)
            final, fwd2 = W.server_flush([g], False, pct)
            byname = {m.name: m.value for m in final}
            assert fwd2 == []
            assert [byname["a.b.c.%dpercentile" % int(p * 100)] for p in pct] == [exp.quantile(p) for p in pct]
            assert [round(byname["a.b.c.%dpercentile" % int(p * 100)], 9) for p in pct] == [6.0, 42.375, 97.7]
            assert byname["s"] == 1.0
            assert "a.b.c.count" not in byname  # imported digests carry no Local* weight
        finally:
            g.close()
        # local-only histogram on a local veneur: 3 aggregates + 3 percentiles
        for v in vals:
            w.ProcessMetric(W.UDPMetric(K("a.b.c", "histogram"), v, scope=W.MetricScope.LocalOnly))
        final, fwd = W.server_flush([w], True, pct)
        assert len(final) == 6 and fwd == []
        # global veneur flush of the same samples
        for v in vals:
            w.ProcessMetric(W.UDPMetric(K("a.b.c", "histogram"), v, scope=W.MetricScope.LocalOnly))
        final, _ = W.server_flush([w], False, pct)
        byname = {m.name: m.value for m in final}
        assert len(final) == 6 and byname["a.b.c.max"] == 100.0 and byname["a.b.c.50percentile"] == 6.0
    finally:
        w.close()


def test_import_chunk_batches_per_class_and_skips_bad_payloads(caplog):
    """Server.ImportMetrics' chunk (http.go:52-67) reaches the engine as one call per class; a
    payload that fails to decode is skipped alone (worker.go:246-266 logs and continues)."""
    w = cpu_worker()
    ms = [W.JSONMetric(K("h%d" % i, "histogram"), [], b"gob%d" % i) for i in range(5)]
    ms += [W.JSONMetric(K("c%d" % i, "counter"), [], struct.pack("<q", i)) for i in range(3)]
    ms += [W.JSONMetric(K("bad", "counter"), [], b"xx")]
    W.import_metrics([w], ms)
    names = [c[0] for c in w.engine.calls]
    assert names.count("import_histos") == 1 and names.count("import_counters") == 1
    assert [c for c in w.engine.calls if c[0] == "import_histos"][0][1] == [0, 1, 2, 3, 4]
    assert "payload is 2 bytes" in caplog.text
    w2 = cpu_worker()
    ms2 = [W.JSONMetric(K("h%d" % i, "histogram"), [], b"bad" if i == 2 else b"ok") for i in range(4)]
    W.import_metrics([w2], ms2)
    ok = [c[1] for c in w2.engine.calls if c[0] == "import_histos"]
    assert ok == [[0], [1], [3]]  # the failing batch retried one by one, the bad one skipped
    assert "Could not merge histograms" in caplog.text
    assert w2.imported == 4


def test_flush_reports_worker_self_metrics():  # worker.go:286-295
    w = cpu_worker()
    w.ProcessMetric(W.UDPMetric(K("a", "counter"), 1.0))
    w.ProcessMetric(W.UDPMetric(K("b", "counter"), 2.0))
    w.ImportMetric(W.JSONMetric(K("c", "counter"), [], struct.pack("<q", 9)))
    w.Flush()
    calls = w.stats.calls
    assert [c[:2] for c in calls] == [("timing", "flush.worker_duration_ns"),
                                     ("count", "worker.metrics_processed_total"),
                                     ("count", "worker.metrics_imported_total")]
    assert calls[0][2] > 0 and calls[0][3] is None and calls[0][4] == 1.0
    assert calls[1][2:] == (2, [], 1.0) and calls[2][2:] == (1, [], 1.0)
    assert w.processed == 0 and w.imported == 0
    w.Flush()  # an empty window reports zeros
    assert calls[-2][2] == 0 and calls[-1][2] == 0


def test_flush_self_metrics_through_a_statsd_client():
    class Client:
        def __init__(self):
            self.seen = []

        def TimeInMilliseconds(self, name, value, tags, rate):
            self.seen.append(name)

        def Count(self, name, value, tags, rate):
            self.seen.append((name, value))

    c = Client()
    w = W.Worker(engine=RecordingEngine(), batch_records=1000, stats=c)
    w.ProcessMetric(W.UDPMetric(K("a", "counter"), 1.0))
    w.Flush()
    assert c.seen == ["flush.worker_duration_ns", ("worker.metrics_processed_total", 1),
                      ("worker.metrics_imported_total", 0)]


def test_counter_gauge_payload_longer_than_8_bytes():  # binary.Read takes the first 8 (samplers.go:171-183)
    w = cpu_worker()
    w.ImportMetric(W.JSONMetric(K("c", "counter"), [], struct.pack("<q", 7) + b"\x99"))
    w.ImportMetric(W.JSONMetric(K("g", "gauge"), [], struct.pack("<d", 2.5) + b"\x01\x02"))
    w.import_chunk([W.JSONMetric(K("c", "counter"), [], struct.pack("<q", 5) + b"\x00")])
    imp = [c for c in w.engine.calls if c[0].startswith("import")]
    assert imp == [("import_counters", [0], [7]), ("import_gauges", [0], [2.5]), ("import_counters", [0], [5])]
    assert w.Flush().global_counters[K("c", "counter")].value == 12


def test_rejected_batch_is_dropped_not_resubmitted(caplog):
    class Rejecting(RecordingEngine):
        def ingest(self, **kw):
            self.calls.append(("ingest",))
            raise EngineError("slot out of range (rc=-1)")

    w = W.Worker(engine=Rejecting(), batch_records=2)
    for i in range(5):
        w.ProcessMetric(W.UDPMetric(K("a%d" % i, "counter"), 1.0))
    # batches of 2 rejected twice; the fifth record still staged, the stage never grows past 2;
    # counted as refused batches, apart from the per-record NaN-rate drops
    assert w.dropped_batches == 2 and w.dropped_batch_records == 4 and w.dropped == 0
    assert w._staged == 1 and "dropping a batch" in caplog.text
    w.Flush()
    assert w.dropped_batches == 3 and w.dropped_batch_records == 5
    assert [c[0] for c in w.engine.calls].count("ingest") == 3


def test_invalid_records_screened_so_valid_batch_mates_are_kept():
    """a NaN-rate record is dropped alone before staging (the engine would refuse the
    whole batch), a NaN / Inf histogram value raises as Add panics -- the valid records staged
    beside them reach the engine."""
    w = W.Worker(engine=RecordingEngine(), batch_records=4)
    w.ProcessMetric(W.UDPMetric(K("c", "counter"), 1.0))
    w.ProcessMetric(W.UDPMetric(K("h", "histogram"), 2.0, sample_rate=float("nan")))
    with pytest.raises(ValueError):
        w.ProcessMetric(W.UDPMetric(K("h", "histogram"), float("inf")))
    w.ProcessMetric(W.UDPMetric(K("h", "histogram"), 3.0))
    w.Flush()
    ing = [c for c in w.engine.calls if c[0] == "ingest"]
    assert len(ing) == 1 and w.dropped == 1 and w.dropped_batches == 0


# ---------------------------------------------------------------- engines in turn (Worker.Flush)
class SlowEngine(RecordingEngine):
    """A RecordingEngine whose flush takes `delay` seconds and which asserts that it never takes
    records while its flush runs."""

    def __init__(self, name, delay, log, **kw):
        super().__init__(**kw)
        self.name, self.delay, self.log, self.busy = name, delay, log, False

    def ingest(self, **kw):
        assert not self.busy, "engine %d took records during its flush" % self.name
        self.log.append(("ingest", self.name))
        super().ingest(**kw)

    def import_counters(self, slot, v):
        assert not self.busy
        super().import_counters(slot, v)

    def flush(self, histo_quantile_mask=None, set_estimate_mask=None):
        self.busy = True
        import time as _t
        _t.sleep(self.delay)
        self.log.append(("flush", self.name))
        out = super().flush(histo_quantile_mask, set_estimate_mask)
        self.busy = False
        return out


def test_worker_engines_in_turn_flush_returns_at_once():
    """Worker(engines=D): Flush swaps the window out (worker.go:276-284) and returns a
    PendingWorkerMetrics at once; window i runs on engine i % D; an engine takes records again
    only after its flush; each window's maps hold that window's values."""
    import time as _t
    log = []
    D, delay = 3, 0.3
    w = W.Worker(engines=[SlowEngine(k, delay, log) for k in range(D)], batch_records=1000)
    wms, returns = [], []
    for i in range(7):
        w.ProcessMetric(W.UDPMetric(K("a", "counter"), float(i + 1)))
        w.ProcessMetric(W.UDPMetric(K("b%d" % i, "counter"), 10.0, sample_rate=0.5))
        w.ImportMetric(W.JSONMetric(K("g", "counter"), [], struct.pack("<q", 100 + i)))
        t0 = _t.perf_counter()
        wms.append(w.Flush())
        returns.append(_t.perf_counter() - t0)
    # the first D flushes find their engines idle: they return before any flush has finished
    assert max(returns[:D]) < delay / 2, returns
    assert all(isinstance(m, W.PendingWorkerMetrics) for m in wms)
    for i, wm in enumerate(wms):
        assert wm.counters[K("a", "counter")].value == i + 1
        assert wm.counters[K("b%d" % i, "counter")].value == 20
        assert wm.global_counters[K("g", "counter")].value == 100 + i
        assert len(wm) == 3
    ing = [n for what, n in log if what == "ingest"]
    assert ing == [i % D for i in range(7)]
    w.close()
    assert w.stats.calls[1] == ("count", "worker.metrics_processed_total", 2, [], 1.0)


def test_worker_flush_raw_in_turn_and_server_flush():
    """flush_raw(copy=True) under rotation is a Future of the window's FlushOutput; server_flush
    over a rotating Worker still yields each window's InterMetrics."""
    log = []
    w = W.Worker(engines=[SlowEngine(k, 0.05, log) for k in range(2)], batch_records=1000)
    futs = []
    for i in range(4):
        w.process_batch(counters=(np.array([0, 1], np.uint32), np.array([i, 2 * i], np.float64),
                                  np.ones(2, np.float32)))
        futs.append(w.flush_raw(copy=True))
    for i, f in enumerate(futs):
        out = f.result()
        assert out.counter_value.tolist() == [i, 2 * i]
    w.ProcessMetric(W.UDPMetric(K("x", "counter"), 4.0))
    final, fwd = W.server_flush([w], False, (0.5,))
    assert [(m.name, m.value) for m in final] == [("x", 4.0)]
    w.close()


def test_worker_drains_at_class_cap_and_pieces_imports():
    """a class's staged records never exceed the engine's max_class_records (the engine
    refuses such a call), and import_chunk sends each class in pieces of at most its cap."""
    class Capped(RecordingEngine):
        max_batch_records = 8
        max_class_records = (2, 8, 8, 3)
        max_batch_member_bytes = 1 << 10

        def ingest(self, **kw):
            for c, k in enumerate(("counters", "gauges", "histos", "sets")):
                if k in kw:
                    assert len(kw[k][0]) <= self.max_class_records[c], (k, len(kw[k][0]))
            super().ingest(**kw)

        def import_counters(self, slot, v):
            assert len(slot) <= self.max_class_records[0]
            super().import_counters(slot, v)

        def import_sets(self, slot, p):
            assert len(slot) <= self.max_class_records[3]
            super().import_sets(slot, p)

    w = W.Worker(engine=Capped(), batch_records=1 << 16)
    assert w.batch_records == 8 and w.class_records == (2, 8, 8, 3)
    for i in range(5):
        w.ProcessMetric(W.UDPMetric(K("c", "counter"), 1.0))
    assert w._staged == 1  # drained at 2 and 4
    for i in range(7):
        w.ProcessMetric(W.UDPMetric(K("s", "set"), "m%d" % i))
    w.import_chunk([W.JSONMetric(K("c%d" % i, "counter"), [], struct.pack("<q", i)) for i in range(5)] +
                   [W.JSONMetric(K("s%d" % i, "set"), [], b"x") for i in range(7)])
    calls = [c[0] for c in w.engine.calls]
    assert calls.count("import_counters") == 3 and calls.count("import_sets") == 3
    assert w.Flush().counters[K("c", "counter")].value == 5


def test_engine_with_pipeline_is_refused():
    with pytest.raises(ValueError):
        W.Worker(engine=RecordingEngine(), pipeline=3)


def test_failed_flush_on_a_flush_thread_is_raised_when_its_engine_is_reused(caplog):
    """D = 2: a flush that fails on its flush thread is raised (and counted) by the next call that
    would hand that engine new records, instead of the window silently staying unflushed."""
    class Failing(RecordingEngine):
        def flush(self, *a, **k):
            raise EngineError("hip error (rc=-3)")
    bad, good = Failing(), RecordingEngine()
    w = W.Worker(engines=[bad, good], batch_records=1000)
    try:
        key = W.MetricKey("a", "counter", "")
        w.ProcessMetric(W.UDPMetric(key, 1.0, tags=[]))
        fut = w.Flush()              # engine 0's flush fails on its thread
        w.ProcessMetric(W.UDPMetric(key, 2.0, tags=[]))
        w.Flush()                    # engine 1
        with pytest.raises(EngineError):
            w.ProcessMetric(W.UDPMetric(key, 3.0, tags=[]))
            w.Flush()                # back to engine 0: its failed flush surfaces here
        assert w.flush_errors == 1
        with pytest.raises(EngineError):
            fut.wait()
    finally:
        w.close()
