"""GPU parity of the device intake (csrc/intake.hip): DogStatsD datagrams parsed and Upserted on
the GPU (DeviceWorker.handle_packets) against the host path of the same text -- the Python mirror
of ParseMetric / HandleMetricPacket (read_metric_datagram, server.go:693-722) feeding
Worker.ProcessMetric (worker.go:187-227) -- compared through Worker.Flush: the same keys in the
same ten maps with the same tags, and bit-identical counters, gauges, set estimates, histogram
local min / max / weight and quantiles (sums within 1e-12: the two paths group
the records into different ingest batches).  Also: imports (ImportMetric's Upsert) sharing the device key
table, NaN sample rates dropped one record at a time, a capacity overflow that leaves the window
unchanged, and a second window after Flush."""
import struct

import numpy as np
import pytest

from veneur_amd import parser as P
from veneur_amd import worker as W

CAP = (2048, 2048, 2048, 2048)
PCT = (0.5, 0.9, 0.99)


def gen_datagrams(rng, n_lines, per=40):
    types = [b"c", b"g", b"h", b"ms", b"s"]
    scope = [b"", b"veneurlocalonly", b"veneurglobalonly", b"veneurglobalonly:1"]
    names = [b"api.req.%d" % i for i in range(25)] + [b"db.q\xc3\xa9", b"n\xff"]
    lines = []
    for i in range(n_lines):
        name = names[int(rng.integers(0, len(names)))]
        t = types[int(rng.integers(0, 5))]
        v = b"u%d" % rng.integers(0, 400) if t == b"s" else b"%.4f" % rng.lognormal(2, 1)
        line = name + b":" + v + b"|" + t
        r = rng.random()
        if r < 0.1:
            line += b"|@0.5"
        elif r < 0.12:
            line += b"|@nan"
        tags = [b"env:%d" % rng.integers(0, 2), b"zone:a"]
        sc = scope[int(rng.integers(0, 4))]
        if sc:
            tags.append(sc)
        if rng.random() < 0.8:
            rng.shuffle(tags)
            line += b"|#" + b",".join(tags)
        if rng.random() < 0.03:
            line = line.replace(b":", b"", 1)  # a parse error
        lines.append(line)
    return [b"\n".join(lines[i:i + per]) for i in range(0, len(lines), per)]


def assert_same(wa, wb):
    for m in W._MAPS:
        a, b = getattr(wa, m), getattr(wb, m)
        assert set(a) == set(b), (m, set(a) ^ set(b))
        for k in a:
            x, y = a[k], b[k]
            assert x.tags == y.tags, (m, k)
            if isinstance(x, (W.Counter, W.Gauge)):
                assert struct.pack("<d", float(x.value)) == struct.pack("<d", float(y.value)), (m, k)
            elif isinstance(x, W.Set):
                assert (x.estimate, x.sparse) == (y.estimate, y.sparse), (m, k)
            else:
                sx = (x.local_weight, x.local_min, x.local_max)
                sy = (y.local_weight, y.local_min, y.local_max)
                assert np.array_equal(np.array(sx).view(np.uint64), np.array(sy).view(np.uint64)), (m, k)
                # the float sums are compensated but batch-grouped: <= 1e-12 relative, as in every parity test
                for u, v in ((x.local_sum, y.local_sum), (x.local_reciprocal_sum, y.local_reciprocal_sum)):
                    assert abs(u - v) <= 1e-12 * abs(v), (m, k, u, v)
                for p in PCT:
                    qx, qy = x.quantile(p), y.quantile(p)
                    assert qx == qy or (qx != qx and qy != qy), (m, k, p)


def workers():
    from veneur_amd.intake import DeviceWorker
    return (W.Worker(capacity=CAP, percentiles=PCT, batch_records=1 << 12),
            DeviceWorker(capacity=CAP, percentiles=PCT, batch_records=1 << 12, intake_bytes=1 << 20))


@pytest.mark.gpu
def test_intake_matches_host_worker():
    rng = np.random.default_rng(21)
    host, dev = workers()
    try:
        errs = 0
        for d in gen_datagrams(rng, 6000):
            errs += len(P.read_metric_datagram([host], d))
            st = dev.handle_packets(d)
        assert dev.parse_errors == errs and dev.processed == host.processed and dev.dropped == host.dropped > 0
        assert_same(host.Flush(), dev.Flush())
        # a second window restarts the slots
        for d in gen_datagrams(rng, 1500):
            P.read_metric_datagram([host], d)
            dev.handle_packets(d)
        assert_same(host.Flush(), dev.Flush())
    finally:
        host.close()
        dev.close()


@pytest.mark.gpu
def test_intake_with_imports_shares_the_key_table():
    rng = np.random.default_rng(22)
    host, dev = workers()
    try:
        imports = [W.JSONMetric(W.MetricKey("api.req.%d" % i, "counter", "env:0,zone:a"), ["env:0", "zone:a"],
                                struct.pack("<q", 1000 + i)) for i in range(0, 25, 3)]
        imports += [W.JSONMetric(W.MetricKey("imp.g%d" % i, "gauge", ""), [], struct.pack("<d", 2.5 * i))
                    for i in range(4)]
        dgs = gen_datagrams(rng, 3000)
        for j, d in enumerate(dgs):
            P.read_metric_datagram([host], d)
            dev.handle_packets(d)
            if j % 20 == 5:
                host.import_chunk(imports)
                dev.import_chunk(imports)
        # a host UDPMetric through the device table too
        m = P.ParseMetric(b"api.req.3:7|c|#env:1,zone:a")
        host.process_metric(m)
        dev.process_metric(m)
        assert_same(host.Flush(), dev.Flush())
    finally:
        host.close()
        dev.close()


@pytest.mark.gpu
def test_intake_capacity_overflow_leaves_window_unchanged():
    from veneur_amd.intake import DeviceWorker
    host = W.Worker(capacity=(8, 8, 8, 8), percentiles=PCT, batch_records=1 << 10)
    dev = DeviceWorker(capacity=(8, 8, 8, 8), percentiles=PCT, batch_records=1 << 10, intake_bytes=1 << 16)
    try:
        ok = b"\n".join(b"c%d:1|c" % i for i in range(5))
        P.read_metric_datagram([host], ok)
        dev.handle_packets(ok)
        with pytest.raises(OverflowError):
            dev.handle_packets(b"\n".join(b"d%d:2|c" % i for i in range(6)))  # 5 + 6 > 8 counters
        assert_same(host.Flush(), dev.Flush())
    finally:
        host.close()
        dev.close()
