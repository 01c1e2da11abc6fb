"""DogStatsD metric-packet parsing (samplers/parser.go:186-307) in front of Worker.ProcessMetric.

The reference's parser_test.go:392-515 cases (types, tags, sample rates, the invalid-packet
table with its error texts, the local/global-only escape tags), the routing KAT of
http_test.go:43-57 (ParseMetric digest == the import hash of the same key), Go's ParseFloat
syntax and float32 rounding of the sample rate, and ReadMetricSocket's newline splitting into
workers (server.go:612-722) with the recording stand-in engine of test_worker.py.
"""
import numpy as np
import pytest

from tests.test_worker import cpu_worker
from veneur_amd import parser as P
from veneur_amd import worker as W

K = W.MetricKey


@pytest.mark.parametrize("packet,typ", [(b"a.b.c:1|c", "counter"), (b"a.b.c:1|g", "gauge"),
                                        (b"a.b.c:1|h", "histogram"), (b"a.b.c:1|ms", "timer")])
def test_parser_types(packet, typ):  # parser_test.go:392-422
    m = P.ParseMetric(packet)
    assert (m.key.name, m.value, m.key.type, m.sample_rate) == ("a.b.c", 1.0, typ, np.float32(1.0))


def test_parser_set_tags_and_rates():  # parser_test.go:424-473
    m = P.ParseMetric(b"a.b.c:foo|s")
    assert (m.value, m.key.type) == ("foo", "set")
    m = P.ParseMetric(b"a.b.c:1|c|#foo:bar,baz:gorch")
    assert m.tags == ["baz:gorch", "foo:bar"] and m.key.joined_tags == "baz:gorch,foo:bar"
    m = P.ParseMetric(b"a.b.c:1|c|@0.1")
    assert m.sample_rate == np.float32(0.1) and m.sample_rate.dtype == np.float32
    P.ParseMetric(b"a.b.c:1|g|@0.1")
    m = P.ParseMetric(b"a.b.c:1|c|@0.1|#foo:bar,baz:gorch")
    assert m.sample_rate == np.float32(0.1) and len(m.tags) == 2
    with pytest.raises(P.ParseError, match="Invalid number"):
        P.ParseMetric(b"a.b.c:fart|c")


INVALID = {  # parser_test.go:475-499
    b"foo": "1 colon", b"foo:1": "1 pipe", b"foo:1||": "metric type", b"foo:|c|": "metric value",
    b"this_is_a_bad_metric:nan|g|#shell": "metric value", b"this_is_a_bad_metric:NaN|g|#shell": "metric value",
    b"this_is_a_bad_metric:-inf|g|#shell": "metric value", b"this_is_a_bad_metric:+inf|g|#shell": "metric value",
    b"foo:1|foo|": "Invalid type", b"foo:1|c||": "pipes", b"foo:1|c|foo": "unknown section",
    b"foo:1|c|@-0.1": ">0", b"foo:1|c|@1.1": "<=1", b"foo:1|c|@0.5|@0.2": "multiple sample rates",
    b"foo:1|c|#foo|#bar": "multiple tag sections",
}


@pytest.mark.parametrize("packet", sorted(INVALID))
def test_invalid_packets(packet):
    with pytest.raises(P.ParseError) as e:
        P.ParseMetric(packet)
    assert INVALID[packet] in str(e.value)


def test_scope_escape_tags():  # parser_test.go:501-515
    m = P.ParseMetric(b"a.b.c:1|h|#veneurlocalonly,tag2:quacks")
    assert m.scope == W.MetricScope.LocalOnly and m.tags == ["tag2:quacks"]
    m = P.ParseMetric(b"a.b.c:1|h|#veneurglobalonly,tag2:quacks")
    assert m.scope == W.MetricScope.GlobalOnly and m.tags == ["tag2:quacks"]
    # only the first escape tag (in sorted order) is removed, and it is not part of the digest
    m = P.ParseMetric(b"a:1|c|#veneurlocalonly,veneurglobalonly")
    assert m.scope == W.MetricScope.GlobalOnly and m.tags == ["veneurlocalonly"]
    assert m.digest == W.metric_digest(K("a", "counter", "veneurlocalonly"))


def test_digest_matches_import_hash():  # http_test.go:43-57
    m = P.ParseMetric(b"foo:1|h|#bar")
    assert m.digest == W.metric_digest(m.key) and m.digest % 96 == W.metric_digest(K("foo", "histogram", "bar")) % 96
    assert P.ParseMetric(b"foo:1|h").digest == W.metric_digest(K("foo", "histogram", ""))


def test_go_parse_float_rules():
    for ok, v in ((b"1.", 1.0), (b".5", 0.5), (b"+2e3", 2000.0), (b"-0", -0.0), (b"1e-400", 0.0)):
        assert P.go_parse_float64(ok) == v
    for bad in (b"1_0", b"0x10", b" 1", b"1 ", b"", b".", b"1e", b"e5", b"+nan", b"1e400"):
        with pytest.raises(P.ParseError):
            P.go_parse_float64(bad)
    # ParseFloat(s, 32) rounds the decimal once: a value just above the float32 midpoint between
    # 1 and 1+2^-23 goes up, although its nearest float64 is the midpoint itself (ties to even -> 1)
    mid_plus = b"1.00000005960464477539062500000000001"
    assert np.float64(float(mid_plus)) == 1 + 2.0 ** -24 and np.float32(float(mid_plus)) == np.float32(1)
    assert P.go_parse_float32(mid_plus) == np.float32(1 + 2.0 ** -23)
    with pytest.raises(P.ParseError):
        P.go_parse_float32(b"3.5e38")
    assert P.go_parse_float32(b"1e-99999999999") == 0
    # NaN passes the (0, 1] check in Go; Inf does not
    assert np.isnan(P.ParseMetric(b"a:1|c|@nan").sample_rate)
    with pytest.raises(P.ParseError, match="<=1"):
        P.ParseMetric(b"a:1|c|@inf")


def test_datagram_to_workers():  # server.go:612-722
    ws = [cpu_worker() for _ in range(3)]
    lines = [b"c%d:%d|c|@0.5|#env:a" % (i % 5, i) for i in range(40)] + [b"", b"bad", b"_e{1,1}:a|b"]
    errs = P.read_metric_datagram(ws, b"\n".join(lines))
    assert len(errs) == 2  # the empty packet is ignored; the event is not on this path
    got = {}
    for i, w in enumerate(ws):
        for k, c in w.Flush().counters.items():
            assert W.metric_digest(k) % 3 == i and k.joined_tags == "env:a"
            got[k.name] = c.value
    assert got == {"c%d" % j: sum(2 * i for i in range(40) if i % 5 == j) for j in range(5)}


@pytest.mark.gpu
def test_gpu_dogstatsd_text_through_worker_matches_oracle():
    """DogStatsD datagrams -> read_metric_datagram -> Worker on the engine, against the restated
    Go worker fed with the generator's own values (not the parser's)."""
    import oracle
    from tests.test_worker import feed
    rng = np.random.default_rng(5)
    types = {"counter": b"c", "gauge": b"g", "histogram": b"h", "timer": b"ms", "set": b"s"}
    scope_tag = {W.MetricScope.MixedScope: b"", W.MetricScope.LocalOnly: b",veneurlocalonly",
                 W.MetricScope.GlobalOnly: b",veneurglobalonly"}
    keys = [("m%d" % i, t, W.MetricScope(int(rng.integers(0, 3)))) for i, t in enumerate(list(types) * 6)]
    cls_of = {"counter": 0, "gauge": 1, "histogram": 2, "timer": 2, "set": 3}
    w = W.Worker(capacity=(64, 64, 64, 64), percentiles=(0.5, 0.9, 0.99), batch_records=4096)
    o = oracle.Worker(64, 64, 64, 64)
    slots, nxt = {}, [0, 0, 0, 0]
    try:
        lines = []
        for _ in range(3000):
            name, typ, sc = keys[int(rng.integers(0, len(keys)))]
            rtxt = [b"1", b"0.5", b"0.1"][int(rng.integers(0, 3))]
            if typ == "set":
                v = "u%d" % rng.integers(0, 500)
                vtxt = v.encode()
            else:
                vtxt = b"%.3f" % rng.lognormal(3, 1)
                v = float(vtxt)
            lines.append(b"%s:%s|%s|@%s|#zone:b,env:a%s" % (name.encode(), vtxt, types[typ], rtxt, scope_tag[sc]))
            k = K(name, typ, "env:a,zone:b")
            mp = W._map_for(typ, sc)
            if (mp, k) not in slots:
                slots[(mp, k)] = nxt[cls_of[typ]]
                nxt[cls_of[typ]] += 1
            feed(o, cls_of[typ], slots[(mp, k)], v, float(np.float32(float(rtxt))))
        for i in range(0, len(lines), 25):  # datagrams of 25 lines
            assert P.read_metric_datagram([w], b"\n".join(lines[i:i + 25])) == []
        wm = w.Flush()
        for (mp, k), s in slots.items():
            smp = getattr(wm, mp)[k]
            cls = cls_of[k.type]
            if cls == 0:
                assert smp.value == o.counter_value(s)
            elif cls == 1:
                assert smp.value == o.gauge_value(s)
            elif cls == 2:
                assert (smp.local_weight, smp.local_min, smp.local_max) == tuple(o.histo_stats(s)[:3])
                assert smp.quantile(0.99) == o.histo_quantile(s, 0.99)
            else:
                assert smp.estimate == o.set_estimate(s)
            assert smp.tags == ["env:a", "zone:b"]
    finally:
        w.close()


def _mutations(rng, n):
    base = [b"a.b.c:1|c", b"x:2.5|g|@0.25|#b:1,a:2", b"t:3e2|ms|#veneurlocalonly,z", b"s:m1|s|#veneurglobalonly",
            b"h:-0.5|h|@1|#", b"q:1.00000005960464477539062500000000001|c|@1.00000005960464477539062500000000001"]
    alphabet = b"|:@#,.e+-0123456789abcghmsnaif\n"
    out = list(INVALID) + base
    for _ in range(n):
        b = bytearray(base[int(rng.integers(0, len(base)))])
        for _ in range(int(rng.integers(1, 4))):
            i = int(rng.integers(0, len(b) + 1))
            op = int(rng.integers(0, 3))
            if op == 0:
                b.insert(i, alphabet[int(rng.integers(0, len(alphabet)))])
            elif op == 1 and i < len(b):
                del b[i]
            elif i < len(b):
                b[i] = alphabet[int(rng.integers(0, len(alphabet)))]
        out.append(bytes(b))
    return out


def test_native_parse_matches_python_mirror():  # vn_parse_dogstatsd vs parse_metric, line by line
    rng = np.random.default_rng(3)
    lines = [l for l in _mutations(rng, 4000) if b"\n" not in l and l]
    got = P.parse_datagram_native(b"\n".join(lines))
    assert len(got) == len(lines)
    for line, g in zip(lines, got):
        try:
            m = P.parse_metric(line) if not line.startswith((b"_e{", b"_sc")) else None
        except P.ParseError:
            m = None
        if m is None:
            assert isinstance(g, int) and g > 0, line
        else:
            assert not isinstance(g, int), (line, g)
            assert (g.key, g.digest, g.scope, g.tags) == (m.key, m.digest, m.scope, m.tags), line
            assert g.sample_rate == m.sample_rate or (np.isnan(g.sample_rate) and np.isnan(m.sample_rate)), line
            assert g.value == m.value or (isinstance(m.value, float) and np.signbit(g.value) == np.signbit(m.value)), line
