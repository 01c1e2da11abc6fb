"""World-size-2 (gloo, CPU) tests of the key-sharded multi-GPU path (veneur_amd.dist).

Rank r owns the keys with FNV-1a digest % N == r (server.go:655 worker routing applied to
GPUs).  Aggregation is per key, so routing a stream by key and flushing every shard on its
own must give exactly the single-consumer flush -- that is the invariant that lets bench.py
run N GPUs with no data-path collective.  The oracle (oracle/) is the checker here; no GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
import veneur_amd as V
from veneur_amd import dist as D

PCT = (0.5, 0.9, 0.99, 0.999)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _streams(d):
    return {k: d[k] for k in ("c_slot", "c_val", "c_rate", "g_slot", "g_val", "h_slot", "h_val", "h_rate",
                              "s_slot", "s_off", "s_bytes")}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    try:
        g = D.Group(backend="gloo")
        full = V.synth(seed=77, n_keys=3000, n_samples=60000)
        mine = D.route_stream(full, rank, world)
        _, _, out = oracle.baseline_run_full(1, full["n_slots"], _streams(mine), PCT)
        # the bench's control plane: max of elapsed, sum of samples
        el = g.max(1.0 + rank)
        tot = g.sum(len(mine["c_slot"]) + len(mine["g_slot"]) + len(mine["h_slot"]) + len(mine["s_slot"]))
        touched = [np.nonzero(t)[0].tolist() for t in out["touched"]]
        res = {"rank": rank, "el": el, "tot": tot, "touched": touched,
               "counter": out["counter"].tolist(), "gauge": out["gauge"].tolist(),
               "histo_q": out["histo_q"].tolist(), "histo_stats": out["histo_stats"].tolist(),
               "set_est": out["set_est"].tolist()}
        allres = g.gather_object(res)
        g.barrier()
        g.close()
        if rank == 0:
            q.put(allres)
    except Exception as ex:  # surface the failure in the parent
        q.put(repr(ex))
        raise


def test_shard_of_matches_reference_routing_kat():
    # http_test.go:31-32: FNV digests % 96 -> 0x4f, 0x3a, 0x2, 0x3c
    digs = [oracle.fnv1a32(b"foo" + b"histogram"), oracle.fnv1a32(b"bar" + b"set"),
            oracle.fnv1a32(b"baz" + b"counter"), oracle.fnv1a32(b"qux" + b"gauge")]
    assert D.shard_of(digs, 96).tolist() == [0x4f, 0x3a, 0x2, 0x3c]


def test_route_stream_partitions_records():
    full = V.synth(seed=5, n_keys=500, n_samples=20000)
    parts = [D.route_stream(full, r, 3) for r in range(3)]
    for sk in ("c_slot", "g_slot", "h_slot", "s_slot"):
        assert sum(len(p[sk]) for p in parts) == len(full[sk])
    for c, sk in enumerate(("c_slot", "g_slot", "h_slot", "s_slot")):
        for r, p in enumerate(parts):
            assert np.all(D.shard_of(full["digest_of_slot"][c][p[sk]], 3) == r)
    # member bytes travel with their records
    p = parts[1]
    full_members = {bytes(full["s_bytes"][full["s_off"][i]:full["s_off"][i + 1]]) for i in range(len(full["s_slot"]))
                    if D.shard_of(full["digest_of_slot"][3][full["s_slot"][i]], 3) == 1}
    got = {bytes(p["s_bytes"][p["s_off"][i]:p["s_off"][i + 1]]) for i in range(len(p["s_slot"]))}
    assert got == full_members


def test_two_rank_sharded_flush_equals_single_consumer():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        allres = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert not isinstance(allres, str), allres
    assert all(p.exitcode == 0 for p in procs)
    assert allres[0]["el"] == 2.0 and allres[1]["el"] == 2.0  # max over ranks

    full = V.synth(seed=77, n_keys=3000, n_samples=60000)
    _, _, ref = oracle.baseline_run_full(1, full["n_slots"], _streams(full), PCT)
    n_total = sum(len(full[k]) for k in ("c_slot", "g_slot", "h_slot", "s_slot"))
    assert allres[0]["tot"] == n_total
    for c in range(4):
        sets = [set(r["touched"][c]) for r in allres]
        assert not (sets[0] & sets[1])                       # disjoint keys: no exchange needed
        assert sets[0] | sets[1] == set(np.nonzero(ref["touched"][c])[0].tolist())
    for r in allres:
        t = r["touched"]
        np.testing.assert_array_equal(np.array(r["counter"])[t[0]], ref["counter"][t[0]])
        np.testing.assert_array_equal(np.array(r["gauge"])[t[1]], ref["gauge"][t[1]])
        np.testing.assert_array_equal(np.array(r["histo_q"])[t[2]], ref["histo_q"][t[2]])
        np.testing.assert_array_equal(np.array(r["histo_stats"])[t[2]], ref["histo_stats"][t[2]])
        np.testing.assert_array_equal(np.array(r["set_est"], dtype=np.uint64)[t[3]], ref["set_est"][t[3]])
