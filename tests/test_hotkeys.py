"""Hot keys spanning ranks: the split-key combine of split.hip restated on CPU (tests/split_protocol.py)
and run by world-size 2 and 3 gloo process groups -- the same protocol the engines run over RCCL.

A hot key's records are dealt round-robin by the key's window arrival index (record j to rank
j % N, veneur_amd.dist.deal).  The owner's combined state is compared with ONE consumer of the
whole ordered stream (the reference: server.go:655 never splits a key):
  counters  exact;  sets  bit-identical registers / b / sparse state;
  histos    within 1e-3 rank error, bit-identical when the key fits the exact prefix.
The GPU counterpart (the engines themselves) is tests/test_split_gpu.py."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

import oracle
from tests import split_protocol as SP
from veneur_amd import dist as D

PCT = (0.5, 0.9, 0.99, 0.999)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream():
    rng = np.random.default_rng(21)
    hs = {}
    hs["h_small"] = np.exp(rng.normal(3.9, 1.0, 3000))        # fits the exact prefix
    hs["h_warm"] = np.exp(rng.normal(3.9, 1.0, 60000))
    hs["h_hot"] = np.exp(rng.normal(3.9, 1.0, 400000))
    rate = {k: np.where(rng.random(len(v)) < 0.1, np.float32(0.5), np.float32(1.0)).astype(np.float32)
            for k, v in hs.items()}
    sets = {}
    sets["s_dense"] = rng.integers(0, 2**64 - 1, 600000, dtype=np.uint64)   # rebases
    u = rng.integers(0, 2**64 - 1, 8300, dtype=np.uint64)
    sets["s_late"] = u[rng.integers(0, 8300, 200000)]                       # switches past J0
    u = rng.integers(0, 2**64 - 1, 50, dtype=np.uint64)
    sets["s_sparse"] = u[rng.integers(0, 50, 90000)]                        # sparse to the end
    ctr = rng.integers(-3, 40, (3, 5000)).astype(np.int64)
    return hs, rate, sets, ctr


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    try:
        g = D.Group(backend="gloo")
        hs, rate, sets, ctr = _stream()
        out = {"rank": rank}
        # counters: each rank's partial sum of its dealt records
        part = np.array([c[D.deal(len(c), world) == rank].sum() for c in ctr], np.int64)
        out["counters"] = SP.counters(g, part).tolist()
        for i, (name, v) in enumerate(sorted(hs.items())):
            mine = D.deal(len(v), world) == rank
            w = (np.float32(1.0) / rate[name][mine]).astype(np.float64)
            td = SP.histo(g, v[mine], w, len(v), owner=i % world)
            if td is not None:
                out[name] = [td.quantile(p) for p in PCT]
        for i, (name, h) in enumerate(sorted(sets.items())):
            mine = D.deal(len(h), world) == rank
            sk = SP.sets(g, h[mine], len(h))
            if i % world == rank:
                out[name] = (sk.sparse, sk.b, sk.registers().tolist() if not sk.sparse else sorted(
                    sk.list_codes().tolist()) + ["tmp"] + sorted(sk.tmp_codes().tolist()), sk.estimate())
        allres = g.gather_object(out)
        g.barrier()
        g.close()
        if rank == 0:
            q.put(allres)
    except Exception as ex:  # surface the failure in the parent
        q.put(repr(ex))
        raise


def _run(world):
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
    got = {}
    for r in allres:
        got.update(r)
    hs, rate, sets, ctr = _stream()
    assert got["counters"] == ctr.sum(axis=1).tolist()
    for name, v in hs.items():
        w = (np.float32(1.0) / rate[name]).astype(np.float64)
        ref = oracle.MergingDigest(100.0)
        ref.add_many(v, w)
        rq = [ref.quantile(p) for p in PCT]
        o = np.argsort(v, kind="stable")
        cw = np.cumsum(w[o])
        F = lambda x: cw[np.searchsorted(v[o], x, side="right") - 1] / cw[-1]
        err = max(abs(F(a) - F(b)) for a, b in zip(got[name], rq))
        assert err <= 1e-3, (name, err)
        if len(v) <= SP.P_HOT:
            assert got[name] == rq, name
    for name, h in sets.items():
        sk = oracle.Sketch()
        for x in h.tolist():
            sk.insert_hash(int(x))
        exp = (sk.sparse, sk.b, sk.registers().tolist() if not sk.sparse else sorted(
            sk.list_codes().tolist()) + ["tmp"] + sorted(sk.tmp_codes().tolist()), sk.estimate())
        assert tuple(got[name]) == exp, name
    assert not got["s_dense"][0] and got["s_dense"][1] >= 1 and got["s_sparse"][0]


def test_split_protocol_two_ranks_gloo():
    _run(2)


def test_split_protocol_three_ranks_gloo():
    _run(3)
