"""Hot keys spanning GPUs (veneur_amd.dist.exchange_hot): a hot key's samples are spread over
every rank, and at flush the partial states meet on the owner rank -- every rank exports its
partial (Histo.Export / Set.Export), one all-gather moves the payloads, the owner imports them
(Histo.Combine / Set.Combine, worker.go:230-268), counters are summed by an all-reduce.

CPU: world-size-2 gloo ranks, each holding its share in the restated Go worker (oracle/) as
the store; the owner's result must equal (a) the reference's global-merge of the two partials
and (b) for sets the single-consumer sketch, for histograms the single-consumer quantiles within
rank-error tolerance.  GPU: the device-resident store (EngineStore) on one GPU, export of one
engine imported into another straight from HBM."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle
from veneur_amd import dist as D

PCT = (0.5, 0.9, 0.99, 0.999)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _identity(payload):
    t = oracle.MergingDigest(100.0)
    t.gob_decode(payload)
    return np.arange(len(t.centroids()[0]), dtype=np.int64)


class OracleStore:
    """exchange_hot's store backed by the restated Go worker (host payload tensors)."""

    def __init__(self, w):
        self.w = w

    def export(self, cls, slots):
        pays = [self.w.histo_gob(int(s)) if cls == "histo" else self.w.set_sketch(int(s)).marshal() for s in slots]
        off = np.zeros(len(pays) + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p in pays])
        buf = torch.from_numpy(np.frombuffer(b"".join(pays) or b"\0", np.uint8).copy())
        return buf[:int(off[-1])], off

    def import_(self, cls, slots, data, off):
        b = data.cpu().numpy().tobytes()
        for s, a, z in zip(slots, off[:-1], off[1:]):
            p = b[int(a):int(z)]
            if cls == "histo":
                assert self.w.import_histo(int(s), p, _identity(p)) == 0
            else:
                assert self.w.import_set(int(s), p) == 0


def _stream(seed=5):
    """4 hot histo keys, 3 hot set keys, 2 hot counters; samples dealt round-robin to 2 ranks."""
    rng = np.random.default_rng(seed)
    nh, ns, nc = 4, 3, 2
    h_slot = rng.integers(0, nh, 60000).astype(np.uint32)
    h_val = np.exp(rng.normal(3.9, 1.0, len(h_slot)))
    h_rate = np.ones(len(h_slot), np.float32)
    s_slot = rng.integers(0, ns, 90000).astype(np.uint32)
    s_hash = rng.integers(0, 2**63, len(s_slot), dtype=np.uint64) * np.uint64(2)
    c_slot = rng.integers(0, nc, 5000).astype(np.uint32)
    c_val = rng.integers(1, 10, len(c_slot)).astype(np.float64)
    c_rate = np.ones(len(c_slot), np.float32)
    return (nh, ns, nc), (h_slot, h_val, h_rate), (s_slot, s_hash), (c_slot, c_val, c_rate)


def _share(arrs, rank, world):
    return tuple(a[rank::world] for a in arrs)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    try:
        g = D.Group(backend="gloo")
        (nh, ns, nc), H, S, Cn = _stream()
        w = oracle.Worker(nc, 1, nh, ns)
        hs = _share(H, rank, world)
        ss = _share(S, rank, world)
        cs = _share(Cn, rank, world)
        w.histo(*hs)
        w.set_hashed(*ss)
        w.counter(*cs)
        store = OracleStore(w)
        h_own = np.arange(nh) % world
        s_own = (np.arange(ns) + 1) % world
        D.exchange_hot(g, store, "histo", np.arange(nh, dtype=np.uint32), h_own)
        D.exchange_hot(g, store, "set", np.arange(ns, dtype=np.uint32), s_own)
        csum = D.allreduce_counters(g, [w.counter_value(s) for s in range(nc)])
        res = {"rank": rank,
               "histo_q": {int(s): [w.histo_quantile(int(s), p) for p in PCT] for s in range(nh) if h_own[s] == rank},
               "set_est": {int(s): int(w.set_estimate(int(s))) for s in range(ns) if s_own[s] == rank},
               "counters": csum.tolist()}
        allres = g.gather_object(res)
        g.barrier()
        g.close()
        if rank == 0:
            q.put(allres)
    except Exception as ex:
        q.put(repr(ex))
        raise


def test_two_rank_hot_key_exchange_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        allres = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert not isinstance(allres, str), allres
    assert all(p.exitcode == 0 for p in procs)
    (nh, ns, nc), H, S, Cn = _stream()
    # (a) the reference's global merge of the partials: owner's partial, then the other's
    parts = []
    for r in range(world):
        w = oracle.Worker(nc, 1, nh, ns)
        w.histo(*_share(H, r, world))
        w.set_hashed(*_share(S, r, world))
        parts.append(w)
    single = oracle.Worker(nc, 1, nh, ns)
    single.histo(*H)
    single.set_hashed(*S)
    single.counter(*Cn)
    got_q, got_s = {}, {}
    for r in allres:
        got_q.update({int(k): v for k, v in r["histo_q"].items()})
        got_s.update({int(k): v for k, v in r["set_est"].items()})
        assert r["counters"] == [single.counter_value(s) for s in range(nc)]
    for s in range(nh):
        own = s % world
        exp = oracle.Worker(nc, 1, nh, ns)
        exp.histo(*_share(H, own, world))
        for r in range(world):
            if r != own:
                p = parts[r].histo_gob(s)
                exp.import_histo(s, p, _identity(p))
        assert got_q[s] == [exp.histo_quantile(s, p) for p in PCT]
        # (b) against one consumer of every sample: merging two half digests costs what a
        # reference global pays for merging its locals' digests (a few 1e-3 of rank); that is
        # the price of splitting a key, which is why only hot keys are split
        vals = np.sort(H[1][H[0] == s])
        F = lambda x: np.searchsorted(vals, x, side="right") / len(vals)
        err = max(abs(F(a) - F(single.histo_quantile(s, p))) for a, p in zip(got_q[s], PCT))
        assert err <= 5e-3, (s, err)
    for s in range(ns):
        own = (s + 1) % world
        exp = oracle.Worker(nc, 1, nh, ns)
        exp.set_hashed(*_share(S, own, world))
        for r in range(world):
            if r != own:
                exp.import_set(s, parts[r].set_sketch(s).marshal())
        assert got_s[s] == exp.set_estimate(s)
        assert got_s[s] == single.set_estimate(s)  # dense, no rebase: the union is exact


@pytest.mark.gpu
def test_engine_store_device_resident_roundtrip():
    """EngineStore on one GPU: export from engine A into a device tensor, import into engine B
    from HBM (vn_import_*_device); B equals the host-path import."""
    import veneur_amd as V
    (nh, ns, nc), H, S, Cn = _stream(7)
    with V.Engine((1, 1, nh, ns), max_batch_records=1 << 17) as a, \
            V.Engine((1, 1, nh, ns), max_batch_records=1 << 17) as b, \
            V.Engine((1, 1, nh, ns), max_batch_records=1 << 17) as c:
        a.ingest(histos=H, set_hashes=S)
        sa = D.EngineStore(a)
        for cls, n in (("histo", nh), ("set", ns)):
            slots = np.arange(n, dtype=np.uint32)
            buf, off = sa.export(cls, slots)
            assert buf.is_cuda
            D.EngineStore(b).import_(cls, slots, buf, off)
            host = bytes(buf.cpu().numpy().tobytes())
            pays = [host[int(off[i]):int(off[i + 1])] for i in range(n)]
            (c.import_histos if cls == "histo" else c.import_sets)(slots, pays)
        fb, fc = b.flush(), c.flush()
    np.testing.assert_array_equal(fb.histo_quantiles, fc.histo_quantiles)
    np.testing.assert_array_equal(fb.set_estimate, fc.set_estimate)
    assert fb.samples_imported == nh + ns
