"""A global veneur over N GPUs (N = 2, gloo on CPU): every rank is handed the same /import bodies
and imports only the keys it owns, digest % N (newJSONMetricsByWorker, http.go:71-139, with the
GPUs as the workers; veneur_amd.dist.route_imports, http_import.handle_import(shard=...)).

Checked here with the restated Go import (oracle Worker.ImportMetric: Histo.Combine,
Set.Combine, counter/gauge Combine) as each rank's merge: every key lands on exactly one rank, in
its arrival order, so the ranks' flushes together are the single consumer's bit for bit -- the
property that lets the GPU import run with no collective.  The GPU engines' own merge of the same
routed chunks is tests/test_import_sharded_gpu.py.
"""
import os
import socket
import struct

import numpy as np
import torch.multiprocessing as mp

import oracle
from veneur_amd import dist as D
from veneur_amd import http_import as H
from veneur_amd import worker as W

K = W.MetricKey
PCT = (0.5, 0.9, 0.99)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def bodies(hosts=6, n_histo=24, n_set=12, seed=3):
    """POST bodies of `hosts` local veneurs (flushForward + PostHelper, deflated), every key from
    every host: digests of a few hundred samples, sketches, global counters and gauges."""
    rng = np.random.default_rng(seed)
    out = []
    for h in range(hosts):
        ms = []
        for k in range(n_histo):
            td = oracle.MergingDigest(100.0)
            n = int(rng.integers(50, 400))
            td.add_many(np.exp(rng.normal(3.0 + 0.05 * k, 1.0, n)), np.where(rng.random(n) < 0.1, 10.0, 1.0))
            ms.append(W.JSONMetric(K("c5.t%d" % k, "timer", "env:p"), ["env:p"], td.gob_encode()))
        for k in range(n_set):
            sk = oracle.Sketch(14)
            for x in rng.integers(0, 2**64 - 1, int(rng.integers(10, 3000)), dtype=np.uint64).tolist():
                sk.insert_hash(int(x))
            ms.append(W.JSONMetric(K("c5.s%d" % k, "set", ""), [], sk.marshal()))
        ms.append(W.JSONMetric(K("c5.c", "counter", ""), [], struct.pack("<q", h + 1)))
        ms.append(W.JSONMetric(K("c5.g", "gauge", ""), [], struct.pack("<d", 0.5 * h)))
        out.append(H.post_body(ms))
    return out


def oracle_import(metrics):
    """The restated Go ImportMetric of `metrics` in order: {key: result}."""
    slots = {}
    for m in metrics:
        slots.setdefault(m.key.type, {}).setdefault(m.key, len(slots.get(m.key.type, {})))
    nh = len(slots.get("timer", {})) + len(slots.get("histogram", {}))
    w = oracle.Worker(max(1, len(slots.get("counter", {}))), max(1, len(slots.get("gauge", {}))), max(1, nh),
                      max(1, len(slots.get("set", {}))))
    for m in metrics:
        s = slots[m.key.type][m.key]
        if m.key.type == "timer":
            assert w.import_histo(s, m.value) == 0
        elif m.key.type == "set":
            w.import_set(s, m.value)
        elif m.key.type == "counter":
            w.import_counter(s, struct.unpack("<q", m.value)[0])
        elif m.key.type == "gauge":
            w.import_gauge(s, struct.unpack("<d", m.value)[0])
    res = {}
    for typ, d in slots.items():
        for key, s in d.items():
            if typ == "timer":
                res[key] = [w.histo_quantile(s, p) for p in PCT] + list(w.histo_stats(s)[5:8])
            elif typ == "set":
                res[key] = w.set_estimate(s)
            elif typ == "counter":
                res[key] = w.counter_value(s)
            else:
                res[key] = w.gauge_value(s)
    return res


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    try:
        g = D.Group(backend="gloo")
        mine = []
        for body, enc in bodies():
            mine += D.route_imports(H.unmarshal_metrics_from_http(body, enc), rank, world)
        res = {(k.name, k.type, k.joined_tags): v for k, v in oracle_import(mine).items()}
        allres = g.gather_object(res)
        g.barrier()
        g.close()
        if rank == 0:
            q.put(allres)
    except Exception as ex:  # surface the failure in the parent
        q.put(repr(ex))
        raise


def test_route_imports_partitions_by_worker_digest():
    ms = [m for body, enc in bodies(hosts=2) for m in H.unmarshal_metrics_from_http(body, enc)]
    for world in (1, 2, 3, 8):
        parts = [D.route_imports(ms, r, world) for r in range(world)]
        assert sum(len(p) for p in parts) == len(ms)
        for r, p in enumerate(parts):
            assert all(W.metric_digest(m.key) % world == r for m in p)
            # arrival order kept inside a rank's share
            idx = [ms.index(m) for m in p]
            assert idx == sorted(idx)
        # the same partition newJSONMetricsByWorker makes over `world` workers
        by = {w: c for c, w in W.json_metrics_by_worker(ms, world)}
        assert all(by.get(r, []) == parts[r] for r in range(world))


def test_sharded_import_two_ranks_gloo_equals_single_consumer():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        allres = q.get(timeout=600)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert not isinstance(allres, str), allres
    assert all(p.exitcode == 0 for p in procs)
    merged = {}
    for r in allres:
        assert not set(r) & set(merged)  # no key on two ranks
        merged.update(r)
    ms = [m for body, enc in bodies() for m in H.unmarshal_metrics_from_http(body, enc)]
    ref = {(k.name, k.type, k.joined_tags): v for k, v in oracle_import(ms).items()}
    assert merged == ref
    assert all(len(r) > 0 for r in allres)  # both ranks own keys


def _routed_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    try:
        g = D.Group(backend="gloo")
        router = D.ImportRouter(g, src=0)
        mine, statuses = [], []
        reqs = bodies() + [(b"[1,2", ""), (b"[]", ""), (b"x", "gzip")]  # + three rejected bodies
        for body, enc in reqs:
            st, part = router.route(body if rank == 0 else None, enc)
            statuses.append(st)
            mine += part
        keys = [(m.key.name, m.key.type, m.key.joined_tags, tuple(m.tags), bytes(m.value)) for m in mine]
        res = {(k.name, k.type, k.joined_tags): v for k, v in oracle_import(mine).items()}
        allres = g.gather_object((router.decoded, statuses, keys, res))
        g.barrier()
        g.close()
        if rank == 0:
            q.put(allres)
    except Exception as ex:  # surface the failure in the parent
        q.put(repr(ex))
        raise


def test_import_router_decodes_each_body_once_two_ranks_gloo():
    """one decode per /import body (on the listener's rank), its JSONMetrics
    routed by digest % N to the ranks as newJSONMetricsByWorker routes them to workers
    (http.go:52-139): each rank's share is route_imports' partition of the decoded body, bit for
    bit, and the ranks' merges together equal the single consumer."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_routed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        allres = q.get(timeout=600)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert not isinstance(allres, str), allres
    assert all(p.exitcode == 0 for p in procs)
    n_bodies = len(bodies()) + 3
    assert [a[0] for a in allres] == [n_bodies, 0]  # every body decoded once, on rank 0 only
    for a in allres:
        assert a[1] == [202] * len(bodies()) + [400, 400, 415]
    ms = [m for body, enc in bodies() for m in H.unmarshal_metrics_from_http(body, enc)]
    for r in range(world):
        want = [(m.key.name, m.key.type, m.key.joined_tags, tuple(m.tags), bytes(m.value))
                for m in D.route_imports(ms, r, world)]
        assert allres[r][2] == want
    merged = {}
    for a in allres:
        assert not set(a[3]) & set(merged)
        merged.update(a[3])
    ref = {(k.name, k.type, k.joined_tags): v for k, v in oracle_import(ms).items()}
    assert merged == ref


def test_pack_metrics_round_trip():
    ms = [W.JSONMetric(K("a\u00e9", "timer", "x:1,y:\ufffd"), ["x:1", "y:\ufffd"], b"\x00\x01"),
          W.JSONMetric(K("", "", ""), [], b""), W.JSONMetric(K("c", "counter", ""), [""], bytes(range(256)))]
    back = D.unpack_metrics(D.pack_metrics(ms))
    assert [(m.key, m.tags, m.value) for m in back] == [(m.key, m.tags, bytes(m.value)) for m in ms]
