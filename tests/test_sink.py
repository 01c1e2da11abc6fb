"""The Datadog sink's flush, native (vn_datadog_flush, csrc/sink.cpp) against its Python restatement
(tests/dd_restated.py over veneur_amd.worker.generate_inter_metrics): request bodies byte for byte.

CPU: the reference's datadog_test.go cases (TestDatadogRate, TestServerTags, TestHostMagicTag,
TestDeviceMagicTag, TestDatadogMetricRouting) and random windows built as flush results by hand --
every map, is_local both ways, all aggregates, names and tags with JSON-escaped and invalid UTF-8
bytes, host:/device:/veneursinkonly: tags, values across the ES6 float cut-offs, NaN quantiles of
empty histograms (a chunk that cannot be encoded), chunking under flushMaxPerBody.
GPU: Worker.flush_datadog on the engine against Worker.Flush + the restatement on the same samples.
"""
import ctypes as C
import json
import math

import numpy as np
import pytest

from tests.dd_restated import datadog_bodies, go_json_float
from veneur_amd import worker as W

TS = 1_700_000_123
ALL_AGG = W.HistogramAggregates(W.Aggregate(127), 7)


class FakeFlush:
    """A vn_flush_result built from numpy arrays (the native side only reads it)."""

    def __init__(self, cls_rows, n_pct):
        import veneur_amd._abi as A
        (cs, cv), (gs, gv), (hs, hst, hq), (ss, se) = cls_rows
        self.keep = [np.ascontiguousarray(a) for a in (cs, cv, gs, gv, hs, hst, hq, ss, se)]
        k = self.keep
        self.r = A.FlushResult(len(k[0]), k[0].ctypes.data_as(A.u32p), k[1].ctypes.data_as(A.i64p),
                               len(k[2]), k[2].ctypes.data_as(A.u32p), k[3].ctypes.data_as(A.f64p),
                               len(k[4]), k[4].ctypes.data_as(A.u32p), k[5].ctypes.data_as(A.f64p),
                               k[6].ctypes.data_as(A.f64p), n_pct, len(k[7]), k[7].ctypes.data_as(A.u32p),
                               k[8].ctypes.data_as(A.u64p), None, 0, 0)


def window(rng, n_keys, engine_pct):
    """Random keys per map, their samplers (WorkerMetrics) and the matching flush result."""
    names = ["api.req", "db.q\u00e9", "a<b>&c", "x\"y\\z", "tab\tnl\n", "bad\udcff", "sep\u2028", "m"]
    tag_pool = ["env:prod", "zone:a", "host:h7", "host:", "device:sda", "veneursinkonly:datadog",
                "veneursinkonly:kafka", "", "k:\u00fc", "t<&>"]
    vals = [0.0, -0.0, 1.0, 10.0, 123.456, 1e-7, 5e-324, 1e21, 9.99e20, 1.5e300, -2.5e-10, 1e-6, 0.1 + 0.2]
    wm = W.WorkerMetrics()
    maps = {m: {} for m in W._MAPS}
    rows = {0: [], 1: [], 2: [], 3: []}
    nxt = [0, 0, 0, 0]
    for i in range(n_keys):
        mp = list(W._MAPS)[int(rng.integers(0, len(W._MAPS)))]
        cls, typ = W._MAPS[mp]
        tags = [tag_pool[int(j)] for j in rng.integers(0, len(tag_pool), int(rng.integers(0, 4)))]
        key = W.MetricKey("%s.%d" % (names[i % len(names)], i), typ, ",".join(tags))
        s = nxt[cls]
        nxt[cls] += 1
        maps[mp][key] = (s, tags)
        touched = rng.random() > 0.1
        v = vals[int(rng.integers(0, len(vals)))] * (1 if rng.random() < 0.5 else float(rng.integers(1, 1000)))
        if cls == 0:
            c = int(rng.integers(-10**12, 10**12)) if touched else 0
            if touched:
                rows[0].append((s, c))
            getattr(wm, mp)[key] = W.Counter(key.name, tags, c, key)
        elif cls == 1:
            g = v if touched else 0.0
            if touched:
                rows[1].append((s, g))
            getattr(wm, mp)[key] = W.Gauge(key.name, tags, g, key)
        elif cls == 3:
            e = int(rng.integers(0, 10**7)) if touched else 0
            if touched:
                rows[3].append((s, e))
            getattr(wm, mp)[key] = W.Set(key.name, tags, e, True, None, key)
        else:
            if touched:
                wgt = float(rng.integers(0, 50))
                st = [wgt, v - 1, v + 1, v * wgt, (1 / v if v else 0.0) * wgt] if wgt else \
                    [0.0, math.inf, -math.inf, 0.0, 0.0]
                q = [v + j for j in range(len(engine_pct))] if wgt else [math.nan] * len(engine_pct)
                rows[2].append((s, st, q))
            else:
                st, q = [0.0, math.inf, -math.inf, 0.0, 0.0], [math.nan] * len(engine_pct)
            getattr(wm, mp)[key] = W.Histo(key.name, tags, *st, dict(zip(engine_pct, q)), None, typ, key)
    # the flush result lists touched slots in ascending order
    cs = sorted(rows[0])
    gs = sorted(rows[1])
    hs = sorted(rows[2], key=lambda r: r[0])
    ss = sorted(rows[3])
    hst = np.zeros((max(1, len(hs)), 8))
    for i, r in enumerate(hs):
        hst[i, :5] = r[1]
    hq = np.array([r[2] for r in hs] or [[0.0] * len(engine_pct)], np.float64).reshape(-1, len(engine_pct))
    ff = FakeFlush(((np.array([r[0] for r in cs], np.uint32), np.array([r[1] for r in cs], np.int64)),
                    (np.array([r[0] for r in gs], np.uint32), np.array([r[1] for r in gs], np.float64)),
                    (np.array([r[0] for r in hs], np.uint32), hst, hq),
                    (np.array([r[0] for r in ss], np.uint32), np.array([r[1] for r in ss], np.uint64))),
                   len(engine_pct))
    return wm, maps, ff


def native(ff, maps, engine_pct, hp, agg, is_local, interval, hostname, tags, mpb):
    from veneur_amd.sink import DatadogSink
    s = DatadogSink(interval, hostname, tags, mpb)
    try:
        return s.bodies(ff.r, maps, engine_pct, hp, agg, is_local, TS)
    finally:
        s.close()


def restated(wm, hp, agg, is_local, interval, hostname, tags, mpb):
    ims = W.generate_inter_metrics([wm], [] if is_local else list(hp), list(hp), agg, is_local, interval)
    return datadog_bodies(ims, interval, hostname, tags, mpb, TS)


@pytest.mark.parametrize("seed", range(6))
def test_random_windows_byte_identical(seed):
    rng = np.random.default_rng(seed)
    engine_pct = (0.5, 0.75, 0.9, 0.99, 0.999)
    hp = [(0.9, 0.99), (0.5, 0.999, 0.75), ()][seed % 3]
    agg = [W.DEFAULT_AGGREGATES, ALL_AGG, W.HistogramAggregates(W.Aggregate(0), 0)][seed % 3]
    for is_local in (False, True):
        wm, maps, ff = window(rng, 300, engine_pct)
        for interval, host, tags, mpb in ((10.0, "h1", ["a:b", "c:d"], 25), (2.5, "", [], 1000), (1.0, "x", ["<&>"], 1)):
            got = native(ff, maps, engine_pct, hp, agg, is_local, interval, host, tags, mpb)
            want = restated(wm, hp, agg, is_local, interval, host, tags, mpb)
            assert got[1] == want[1]
            assert len(got[0]) == len(want[0])
            for (ok_a, a), (ok_b, b) in zip(got[0], want[0]):
                assert ok_a == ok_b and a == b, (a[:300], b[:300])
            for ok, body in got[0]:  # well-formed JSON
                if ok:
                    json.loads(body)


def one_metric(m_type, tags, value=10.0, name="foo.bar.baz"):
    """A window with one counter (or gauge) key: the datadog_test.go fixtures."""
    wm = W.WorkerMetrics()
    mp = "counters" if m_type == "counter" else "gauges"
    key = W.MetricKey(name, m_type, ",".join(tags))
    maps = {m: {} for m in W._MAPS}
    maps[mp][key] = (0, tags)
    cs = (np.array([0], np.uint32), np.array([int(value)], np.int64)) if m_type == "counter" else \
        (np.zeros(0, np.uint32), np.zeros(0, np.int64))
    gs = (np.array([0], np.uint32), np.array([value])) if m_type == "gauge" else (np.zeros(0, np.uint32), np.zeros(0))
    ff = FakeFlush((cs, gs, (np.zeros(0, np.uint32), np.zeros((1, 8)), np.zeros((1, 1))),
                    (np.zeros(0, np.uint32), np.zeros(0, np.uint64))), 1)
    return maps, ff


def series(maps, ff, hostname="somehostname", tags=("a:b", "c:d"), interval=10.0):
    out, _ = native(ff, maps, (0.5,), (), W.DEFAULT_AGGREGATES, False, interval, hostname, list(tags), 15)
    return [m for ok, b in out if ok for m in json.loads(b)["series"]]


def test_datadog_rate_and_server_tags():  # datadog_test.go:28-65
    s = series(*one_metric("counter", ["gorch:frobble", "x:e"]))
    assert s[0]["type"] == "rate" and s[0]["points"][0][1] == 1.0
    assert s[0]["host"] == "somehostname" and "a:b" in s[0]["tags"]
    assert s[0]["tags"] == ["a:b", "c:d", "gorch:frobble", "x:e"] and s[0]["interval"] == 10


def test_host_and_device_magic_tags():  # datadog_test.go:67-105
    s = series(*one_metric("counter", ["gorch:frobble", "host:abc123", "x:e"]), hostname="badhostname")
    assert s[0]["host"] == "abc123" and "host:abc123" not in s[0]["tags"] and "x:e" in s[0]["tags"]
    s = series(*one_metric("counter", ["gorch:frobble", "device:abc123", "x:e"]), hostname="badhostname")
    assert s[0]["device_name"] == "abc123" and "device:abc123" not in s[0]["tags"] and "x:e" in s[0]["tags"]


def test_metric_routing():  # datadog_test.go:203-260
    assert series(*one_metric("counter", ["gorch:frobble", "x:e"]))
    assert series(*one_metric("counter", ["gorch:frobble", "x:e", "veneursinkonly:datadog"]))
    assert not series(*one_metric("counter", ["gorch:frobble", "x:e", "veneursinkonly:kafka"]))


def test_float_encoding_matches_go_rules():
    from veneur_amd.sink import DatadogSink  # noqa: F401
    rng = np.random.default_rng(9)
    xs = [0.0, -0.0, 1e-6, 9.99999e-7, 1e21, 9.999999999999999e20, 1e20, 123456789.0, 0.1, 2.5e-8, -1.5e-300,
          float(np.finfo(np.float64).max), 5e-324, 1.7e9]
    xs += list(rng.standard_normal(500) * 10.0 ** rng.integers(-30, 30, 500))
    xs += [float(x) for x in rng.integers(1, 2**62, 200)]
    for x in xs:
        maps, ff = one_metric("gauge", [], value=x)
        out, _ = native(ff, maps, (0.5,), (), W.DEFAULT_AGGREGATES, False, 10.0, "", [], 15)
        body = out[0][1].decode()
        assert ",%s]]" % go_json_float(x) in body, (x, body)
        assert float(json.loads(body)["series"][0]["points"][0][1]) == x


@pytest.mark.gpu
@pytest.mark.parametrize("is_local", [False, True])
def test_gpu_worker_flush_datadog_matches_restatement(is_local):
    from veneur_amd import parser as P
    from veneur_amd.sink import DatadogSink
    rng = np.random.default_rng(4)
    lines = []
    for i in range(4000):
        t = [b"c", b"g", b"h", b"ms", b"s"][i % 5]
        v = b"u%d" % rng.integers(0, 300) if t == b"s" else b"%.3f" % rng.lognormal(2, 1)
        sc = [b"", b",veneurlocalonly", b",veneurglobalonly"][int(rng.integers(0, 3))]
        lines.append(b"k%d:%s|%s|#env:a,host:h%d%s" % (i % 97, v, t, i % 3, sc))
    dg = b"\n".join(lines)
    pct = (0.5, 0.9, 0.99)
    hp = (0.9, 0.99)
    a = W.Worker(capacity=(4096,) * 4, percentiles=pct)
    b = W.Worker(capacity=(4096,) * 4, percentiles=pct)
    sink = DatadogSink(10.0, "myhost", ["dc:1"], 40)
    try:
        P.read_metric_datagram([a], dg)
        P.read_metric_datagram([b], dg)
        got = b.flush_datadog(sink, hp, ALL_AGG, is_local, timestamp=TS)
        wm = a.Flush(is_local=is_local, need_median=True)
        ims = W.generate_inter_metrics([wm], [] if is_local else list(hp), list(hp), ALL_AGG, is_local, 10.0)
        want = datadog_bodies(ims, 10.0, "myhost", ["dc:1"], 40, TS)
        assert got[1] == want[1] and got[0] == want[0]
    finally:
        sink.close()
        a.close()
        b.close()


def test_large_window_threaded_byte_identical():
    """Enough InterMetrics that the native builder splits them over host threads."""
    rng = np.random.default_rng(77)
    engine_pct = (0.5, 0.9, 0.99)
    wm, maps, ff = window(rng, 20000, engine_pct)
    got = native(ff, maps, engine_pct, (0.9, 0.99), ALL_AGG, False, 10.0, "h", ["a:b"], 700)
    want = restated(wm, (0.9, 0.99), ALL_AGG, False, 10.0, "h", ["a:b"], 700)
    assert got[1] == want[1] and got[1][0] > 50000
    assert got[0] == want[0]
