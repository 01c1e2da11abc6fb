"""A global veneur over two GPUs, in-process on one device: two engines, each handed every /import
body and importing only the keys it owns (http_import.handle_import(shard=(rank, 2)),
digest % 2 as newJSONMetricsByWorker routes, http.go:71-139).  The two flushes together must be
the single consumer's (oracle, the restated Go ImportMetric of every body in order): every timer
quantile bit-identical, set estimates, counter and gauge values exact, and no key on both ranks.
"""
import pytest

from tests.test_import_sharded import PCT, bodies, oracle_import
from veneur_amd import http_import as H
from veneur_amd import worker as W

pytestmark = pytest.mark.gpu


def _results(wm):
    out = {}
    for k, h in wm.timers.items():
        out[(k.name, k.type, k.joined_tags)] = [h.quantile(p) for p in PCT]
    for k, s in wm.sets.items():
        out[(k.name, k.type, k.joined_tags)] = s.estimate
    for m in ("counters", "global_counters", "gauges", "global_gauges"):
        for k, c in getattr(wm, m).items():
            out[(k.name, k.type, k.joined_tags)] = c.value
    return out


def test_sharded_import_two_engines_equals_single_consumer():
    bs = bodies(hosts=8, n_histo=40, n_set=16, seed=9)
    ws = [W.Worker(capacity=(8, 8, 64, 32), percentiles=PCT, batch_records=1 << 16) for _ in range(2)]
    try:
        n = 0
        for body, enc in bs:
            for r, w in enumerate(ws):
                st, k = H.handle_import([w], body, enc, shard=(r, 2))
                assert st == 202
                n += k
        got = [_results(w.Flush()) for w in ws]
    finally:
        for w in ws:
            w.close()
    ms = [m for body, enc in bs for m in H.unmarshal_metrics_from_http(body, enc)]
    assert n == len(ms)
    assert got[0] and got[1] and not set(got[0]) & set(got[1])
    ref = {(k.name, k.type, k.joined_tags): (v[:len(PCT)] if k.type == "timer" else v)
           for k, v in oracle_import(ms).items()}
    merged = {**got[0], **got[1]}
    assert merged == ref
