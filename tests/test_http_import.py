"""POST /import envelope (handlers_global.go:53-206) in front of Worker.ImportMetric.

The CPU tests are the reference's http_test.go:101-253 cases (fixtures/import.deflate and
import.uncompressed accepted; gzip 415; deflate header on plain JSON and plain header on
deflated bytes 400; wrong struct type, slice of empty structs and empty list 400) plus the Go
decoding rules veneur_amd.http_import restates, checked with the recording stand-in engine of
test_worker.py.  The GPU test sends the fixture through handle_import into a Worker on the real
engine and checks the quantiles of the forwarded digest ({1,2,7,8,100}: p50 = 6, p75 = 42.375,
p99 = 97.7, server_test.go:121-138).
"""
import base64
import gzip
import json
import os
import struct
import zlib

import pytest

from tests.test_worker import cpu_worker
from veneur_amd import http_import as H
from veneur_amd import worker as W

GOLD = os.path.join(os.path.dirname(__file__), "golden")
K = W.MetricKey


def fixture(name):
    return open(os.path.join(GOLD, name), "rb").read()


def status(body, enc=""):
    return H.handle_import([cpu_worker()], body, enc)[0]


def test_import_fixtures_accepted():  # http_test.go:123-133
    for name, enc in (("import.deflate", "deflate"), ("import.uncompressed", "")):
        ws = [cpu_worker()]
        assert H.handle_import(ws, fixture(name), enc) == (202, 1)
        assert ("import_histos", [0]) in ws[0].engine.calls
    ms = H.unmarshal_metrics_from_http(fixture("import.deflate"), "deflate")
    assert ms[0].key == K("a.b.c", "histogram", "") and ms[0].tags == []
    assert ms[0].value == fixture("tdigest_1_2_7_8_100.gob")


def test_import_encoding_errors():  # http_test.go:135-211
    plain = fixture("import.uncompressed")
    assert status(gzip.compress(plain), "gzip") == 415
    assert status(plain, "deflate") == 400
    assert status(fixture("import.deflate"), "") == 400
    with pytest.raises(H.ImportRequestError) as e:
        H.unmarshal_metrics_from_http(plain, "br")
    assert (e.value.status, e.value.cause) == (415, "unknown_content_encoding")


def test_import_empty_and_malformed():  # http_test.go:213-253, nonEmpty (handlers_global.go:192-206)
    assert status(json.dumps([{"Bad": "Foo"}, {"Bad": "Bar"}]).encode()) == 400
    assert status(b"[]") == 400
    assert status(b"null") == 400
    assert status(b"[null, {}]") == 400
    assert status(b"") == 400
    assert status(b'{"name": "a"}') == 400  # not an array
    # Go's nil vs empty: an empty tags list or value string is not the zero JSONMetric
    assert status(b'[{"tags": []}]') == 202
    assert status(b'[{"value": ""}]') == 202


def test_import_go_json_rules():
    v = base64.b64encode(struct.pack("<q", 7)).decode()
    body = '  [{"NAME": "c", "Type": "counter", "tagString": "a:b", "TAGS": ["a:b", null], "value": "%s", ' \
           '"extra": {"x": [1, 2]}}] trailing garbage' % v
    (m,) = H.unmarshal_metrics_from_http(body.encode())
    assert m.key == K("c", "counter", "a:b") and m.tags == ["a:b", ""] and m.value == struct.pack("<q", 7)
    # U+212A KELVIN SIGN folds to 'k' and U+017F LONG S to 's' (encoding/json fold.go)
    (m,) = H.unmarshal_metrics_from_http('[{"name": "x", "type": "set", "tag\u017f": ["t"]}]'.encode())
    assert m.tags == ["t"]
    # the last duplicate key wins; null leaves the zero value
    (m,) = H.unmarshal_metrics_from_http(b'[{"name": "a", "name": "b", "type": null, "tagstring": "t"}]')
    assert m.key == K("b", "", "t")
    # base64 with embedded newlines is accepted, without padding it is not
    (m,) = H.unmarshal_metrics_from_http(('[{"name": "a", "value": "%s\\n%s"}]' % (v[:4], v[4:])).encode())
    assert m.value == struct.pack("<q", 7)
    for bad in (b'[{"name": "a", "value": "AAA"}]', b'[{"name": 5}]', b'[{"name": "a", "tags": "x"}]',
                b'[{"name": "a", "value": 5}]', b'[{"name": "a", "tags": [1]}]', b'[3]',
                b'[{"name": "a", "x": NaN}]', b'[{"name": "a"}'):
        with pytest.raises(H.ImportRequestError) as e:
            H.unmarshal_metrics_from_http(bad)
        assert (e.value.status, e.value.cause) == (400, "json"), bad


def test_import_deflate_stream_rules():
    plain = fixture("import.uncompressed")
    z = zlib.compress(plain + b"\n" + b" " * 5000)
    assert len(H.unmarshal_metrics_from_http(z, "deflate")) == 1
    # a bad adler32 trailer is never read: the JSON value completes before it
    assert len(H.unmarshal_metrics_from_http(z[:-4] + b"\0\0\0\0", "deflate")) == 1
    # a stream cut inside the JSON value is an error; so is a header that fails zlib.NewReader
    for bad in (zlib.compress(plain)[:40], b"\x78", b"\x79\x9c" + z[2:], b"\x78\xbb" + z[2:]):
        with pytest.raises(H.ImportRequestError) as e:
            H.unmarshal_metrics_from_http(bad, "deflate")
        assert e.value.status == 400, bad
    # FDICT set with a valid check value (0x7820 % 31 == 0): a preset dictionary nobody supplies
    with pytest.raises(H.ImportRequestError) as e:
        H.unmarshal_metrics_from_http(b"\x78\x20" + z[2:], "deflate")
    assert (e.value.status, e.value.cause) == (400, "deflate")


def test_import_routes_by_digest_and_logs_bad_payloads():  # http.go:52-67, worker.go:246-266
    ms = [{"name": "c%d" % i, "type": "counter", "tagstring": "", "tags": None,
           "value": base64.b64encode(struct.pack("<q", i)).decode()} for i in range(12)]
    ms.append({"name": "bad", "type": "counter", "value": base64.b64encode(b"abc").decode()})
    ms.append({"name": "u", "type": "unknowntype", "value": ""})
    ws = [cpu_worker() for _ in range(3)]
    assert H.handle_import(ws, zlib.compress(json.dumps(ms).encode()), "deflate") == (202, 14)
    got = {}
    for i, w in enumerate(ws):
        assert w.imported == sum(W.metric_digest(K(m["name"], m["type"], "")) % 3 == i for m in ms)
        for k, c in w.Flush().global_counters.items():
            assert W.metric_digest(k) % 3 == i
            got[k.name] = c.value
    # the 3-byte counter payload is logged and skipped after Upsert made its sampler (worker.go:235-250)
    assert got == dict({"c%d" % i: i for i in range(12)}, bad=0)


@pytest.mark.gpu
def test_gpu_import_fixture_through_envelope():  # http_test.go:123-133 + server_test.go:121-138
    import numpy as np

    import oracle
    w = W.Worker(capacity=(64, 64, 64, 64), percentiles=(0.5, 0.75, 0.99), batch_records=4096)
    try:
        assert H.handle_import([w], fixture("import.uncompressed"), "") == (202, 1)
        h = w.Flush().histograms[K("a.b.c", "histogram", "")]
        assert h.quantile(0.5) == 6 and h.quantile(0.75) == 42.375
        assert h.quantile(0.99) == pytest.approx(97.7, rel=1e-15)
        # the same digest forwarded twice (deflated and plain) merges into one key
        assert H.handle_import([w], fixture("import.deflate"), "deflate") == (202, 1)
        assert H.handle_import([w], fixture("import.uncompressed"), "") == (202, 1)
        h = w.Flush().histograms[K("a.b.c", "histogram", "")]
        td = oracle.MergingDigest(100.0)
        td.add_many(np.array([1, 2, 7, 8, 100] * 2, np.float64), np.ones(10))
        for p in (0.5, 0.75, 0.99):
            assert h.quantile(p) == pytest.approx(td.quantile(p), rel=1e-12)
    finally:
        w.close()


def test_forward_body_matches_go_encoder():  # http/http.go:116-170, fixtures/import.uncompressed
    plain = fixture("import.uncompressed")
    ms = H.unmarshal_metrics_from_http(plain)
    assert H.marshal_json_metrics(ms) == plain  # byte-identical to the Go json.Encoder output
    body, enc = H.post_body(ms)
    assert enc == "deflate" and zlib.decompress(body) == plain
    m = W.JSONMetric(K("a<b>&\"\\\n\x01 é", "set", "x:y"), ["x:y"], b"\x00\xff")
    raw = H.marshal_json_metrics([m])
    assert raw == ('[{"name":"a\\u003cb\\u003e\\u0026\\"\\\\\\n\\u0001\\u2028é","type":"set","tagstring":"x:y",'
                   '"tags":["x:y"],"value":"AP8="}]\n').encode()
    assert H.unmarshal_metrics_from_http(raw) == [m]


def test_flush_forward_round_trip_cpu():  # flusher.go:264-353 -> handleImport
    local = cpu_worker()
    local.ProcessMetric(W.UDPMetric(K("c", "counter"), 3.0, scope=W.MetricScope.GlobalOnly))
    local.ProcessMetric(W.UDPMetric(K("c2", "counter"), 4.0))  # mixed counters are not forwarded
    wm = local.Flush()
    ms = H.flush_forward([wm])
    assert [m.key for m in ms] == [K("c", "counter")] and ms[0].value == struct.pack("<q", 3)
    glob = cpu_worker()
    assert H.handle_import([glob], *H.post_body(ms)) == (202, 1)
    assert glob.Flush().global_counters[K("c", "counter")].value == 3


@pytest.mark.gpu
def test_gpu_forward_through_envelope_matches_direct_import():
    """A local Worker flushed with forward=True (device GobEncode / MarshalBinary), its exports
    posted through post_body and handle_import into a global Worker: the global's quantiles and
    set estimates equal those of the same JSONMetrics handed to ImportMetric directly."""
    import numpy as np
    rng = np.random.default_rng(11)
    local = W.Worker(capacity=(64, 64, 64, 64), percentiles=(0.5, 0.9, 0.99), batch_records=4096)
    try:
        for i in range(2000):
            k = int(rng.integers(0, 8))
            local.ProcessMetric(W.UDPMetric(K("h%d" % k, "histogram", "env:a"), float(np.exp(rng.normal(3, 1))),
                                            tags=["env:a"]))
            local.ProcessMetric(W.UDPMetric(K("s%d" % (k % 3), "set"), "m%d" % int(rng.integers(0, 50000))))
            local.ProcessMetric(W.UDPMetric(K("g", "gauge"), float(i), scope=W.MetricScope.GlobalOnly))
        ms = H.flush_forward([local.Flush(forward=True)])
    finally:
        local.close()
    assert len(ms) == 1 + 8 + 3
    res = []
    for via_http in (True, False):
        g = W.Worker(capacity=(64, 64, 64, 64), percentiles=(0.5, 0.9, 0.99), batch_records=4096)
        try:
            if via_http:
                assert H.handle_import([g], *H.post_body(ms)) == (202, len(ms))
            else:
                for m in ms:
                    g.ImportMetric(m)
            wm = g.Flush()
            res.append(({k: [h.quantile(p) for p in (0.5, 0.9, 0.99)] for k, h in wm.histograms.items()},
                        {k: s.estimate for k, s in wm.sets.items()},
                        {k: x.value for k, x in wm.global_gauges.items()}))
        finally:
            g.close()
    assert res[0] == res[1]
    assert res[0][2] == {K("g", "gauge"): 1999.0} and len(res[0][0]) == 8 and len(res[0][1]) == 3
