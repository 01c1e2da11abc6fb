"""Split (hot) keys over a group of engines (include/veneur_amd.h "multi-GPU", split.hip).

A hot key's records are dealt round-robin by the key's window arrival index (record j to rank
j % N); at flush the ranks' partial states meet on the key's owner.  These tests run N engines
on ONE GPU as an in-process group (vn_comm_init_local: each rank's flush in its own host
thread, the same exchange code as RCCL with device-to-device copies for transport) and compare
the owner's result with ONE consumer of the whole stream -- the reference semantics, since veneur
never splits a key (server.go:655 routes every record of a key to one worker):
  counters  bit-exact;
  sets      bit-exact sketch state (registers, b, nz, sparse list / tmpSet) and estimate, through
            the sparse->dense switch and rebase epochs;
  histos    Local* weight/min/max exact, sums 1e-12, quantiles within 1e-3 rank error (and
            bit-exact when the key's window fits the exactly replayed prefix).
"""
import threading

import numpy as np
import pytest

import oracle
import veneur_amd as V
from veneur_amd.engine import Comm
from tests.util import PCT
from tests.util import FAST_ONLY

pytestmark = pytest.mark.gpu


def deal(keys, N):
    """rank of each record: its key's window arrival index j, j % N"""
    keys = np.asarray(keys)
    j = np.zeros(len(keys), np.int64)
    seen = {}
    for i, k in enumerate(keys.tolist()):
        c = seen.get(k, 0)
        j[i] = c
        seen[k] = c + 1
    return j % N, j


def run_group(N, build, cap=(8, 8, 8, 8), split_max=1 << 22, close=False, **kw):
    """N engines in one in-process group; build(rank, engine) feeds a rank; flush in N threads."""
    comms = Comm.local(N)
    engines = [V.Engine(cap, percentiles=PCT, max_batch_records=1 << 20, split_max_records=split_max, **kw)
               for _ in range(N)]
    errs = []
    try:
        for r, e in enumerate(engines):
            e.set_comm(comms[r])
            build(r, e)
        if close:  # every rank's combine starts in the engine's own thread (vn_split_close)
            for e in engines:
                e.split_close()

        def combine(r):
            try:
                engines[r].split_combine()
            except Exception as ex:  # noqa: BLE001
                errs.append(ex)

        th = [threading.Thread(target=combine, args=(r,)) for r in range(N)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=600)
        assert not errs, errs
        states = [[e.read_set(s) for s in range(cap[3])] for e in engines]
        out = [e.flush() for e in engines]  # nothing split left: no collective
        return out, states
    finally:
        for e in engines:
            e.close()
        for c in comms:
            c.close()


@pytest.mark.parametrize("N", [1, 2, 3])
def test_split_counters_exact(N):
    rng = np.random.default_rng(1)
    n = 20000
    keys = rng.integers(0, 3, n).astype(np.uint32)
    vals = rng.integers(-5, 50, n).astype(np.float64)
    rates = np.where(rng.random(n) < 0.2, np.float32(0.1), np.float32(1.0)).astype(np.float32)
    owners = np.array([1 % N, 0, (2 % N)], np.uint32)
    rank, _ = deal(keys, N)

    def build(r, e):
        e.split_keys(0, np.arange(3, dtype=np.uint32) + 2, owners)  # local slots 2, 3, 4
        m = rank == r
        e.ingest(counters=(keys[m] + 2, vals[m], rates[m]))
        e.ingest(counters=(np.array([7], np.uint32), np.array([1.0]), np.array([1.0], np.float32)))  # not split

    out, _ = run_group(N, build)
    w = oracle.Worker(8, 1, 1, 1)
    w.counter(keys + 2, vals, rates)
    for k in range(3):
        o = int(owners[k])
        for r in range(N):
            got = dict(zip(out[r].counter_slot.tolist(), out[r].counter_value.tolist()))
            if r == o:
                assert got[k + 2] == w.counter_value(k + 2)
            else:
                assert k + 2 not in got
    for r in range(N):
        assert dict(zip(out[r].counter_slot.tolist(), out[r].counter_value.tolist()))[7] == 1


def _set_stream(seed):
    """hashed inserts of five split set keys:
    0  ~2.4M distinct: dense, several rebase epochs
    1  ~300k distinct: dense, first rebase
    2  8300 distinct x 36 repeats: switches to dense late (past the first gathered records)
    3  60 distinct x 3000 repeats: sparse through 180k inserts
    4  one insert
    5  7000 distinct x 40 repeats: a ~14 KiB list, sparse to the end
    6  20000 distinct x 5 repeats: switches early"""
    rng = np.random.default_rng(seed)
    parts = []
    parts.append((np.zeros(2_400_000, np.uint32), rng.integers(0, 2**64 - 1, 2_400_000, dtype=np.uint64)))
    parts.append((np.ones(300_000, np.uint32), rng.integers(0, 2**64 - 1, 300_000, dtype=np.uint64)))
    u = rng.integers(0, 2**64 - 1, 8300, dtype=np.uint64)
    parts.append((np.full(300_000, 2, np.uint32), u[rng.integers(0, 8300, 300_000)]))
    u = rng.integers(0, 2**64 - 1, 60, dtype=np.uint64)
    parts.append((np.full(180_000, 3, np.uint32), u[rng.integers(0, 60, 180_000)]))
    parts.append((np.full(1, 4, np.uint32), rng.integers(0, 2**64 - 1, 1, dtype=np.uint64)))
    u = rng.integers(0, 2**64 - 1, 7000, dtype=np.uint64)
    parts.append((np.full(280_000, 5, np.uint32), u[rng.integers(0, 7000, 280_000)]))
    u = rng.integers(0, 2**64 - 1, 20000, dtype=np.uint64)
    parts.append((np.full(100_000, 6, np.uint32), u[rng.integers(0, 20000, 100_000)]))
    keys = np.concatenate([p[0] for p in parts])
    hs = np.concatenate([p[1] for p in parts])
    o = rng.permutation(len(keys))
    return keys[o], hs[o]


@pytest.mark.parametrize("N", [1, 2, 4])
def test_split_sets_bit_exact_through_switch_and_rebase(N):
    keys, hs = _set_stream(5)
    nk = 7
    owners = (np.arange(nk) * 7 + 1) % N
    rank, _ = deal(keys, N)

    def build(r, e):
        e.split_keys(3, np.arange(nk, dtype=np.uint32), owners.astype(np.uint32))
        m = rank == r
        for part in np.array_split(np.nonzero(m)[0], 3):  # several split batches per window
            e.ingest_split(set_hashes=(keys[part], hs[part]))

    out, states = run_group(N, build, cap=(1, 1, 1, 8))
    w = oracle.Worker(1, 1, 1, nk)
    w.set_hashed(keys, hs)
    for k in range(nk):
        o = int(owners[k])
        sk = w.set_sketch(k)
        st = states[o][k]
        assert bool(st["sparse"]) == sk.sparse, k
        assert st["b"] == sk.b, k
        if sk.sparse:
            np.testing.assert_array_equal(st["list"], sk.list_codes())
            np.testing.assert_array_equal(np.sort(st["tmp"]), np.sort(sk.tmp_codes()))
            assert st["list_bytes"] == sk.list_bytes()
        else:
            np.testing.assert_array_equal(st["registers"], sk.registers())
            assert st["nz"] == sk.nz, k
        est = dict(zip(out[o].set_slot.tolist(), out[o].set_estimate.tolist()))
        assert est[k] == w.set_estimate(k), k
        for r in range(N):
            if r != o:
                assert k not in out[r].set_slot.tolist()
    assert w.set_sketch(0).b >= 2 and w.set_sketch(1).b >= 1  # the stream did rebase
    assert w.set_sketch(3).sparse and w.set_sketch(5).sparse and not w.set_sketch(6).sparse


def _histo_stream(seed):
    """timer samples of four split keys: 600k, 80k, 9000 and 3000 samples (the last fits the
    exactly replayed prefix of 4096 window records)"""
    rng = np.random.default_rng(seed)
    sizes = [600_000, 80_000, 9_000, 3_000]
    keys = np.concatenate([np.full(n, k, np.uint32) for k, n in enumerate(sizes)])
    o = rng.permutation(len(keys))
    keys = keys[o]
    vals = np.exp(rng.normal(3.912023005428146, 1.0, len(keys)))
    u = rng.random(len(keys))
    rates = np.where(u < 0.05, np.float32(0.1), np.where(u < 0.1, np.float32(0.5), np.float32(1.0))).astype(np.float32)
    return keys, vals, rates, len(sizes)


def _rank_err(vals, w, q_eng, q_ref):
    o = np.argsort(vals, kind="stable")
    sv, cw = vals[o], np.cumsum(w[o])
    F = lambda q: (cw[np.searchsorted(sv, q, side="right") - 1] / cw[-1]) if np.searchsorted(sv, q, side="right") else 0.0
    return max(abs(F(a) - F(b)) for a, b in zip(q_eng, q_ref))


@pytest.mark.parametrize("N,fast", [(1, False), (2, False), (4, False)] +
                         [pytest.param(n, True, marks=FAST_ONLY) for n in (1, 2, 4)])
def test_split_histos_within_rank_error(N, fast):
    """default (exact) mode: every record of a split key is gathered to its owner in window order
    and replayed, so the owner's quantiles are a single consumer's bit for bit; the opt-in fast
    mode (threshold 32768: a 4096-record exact prefix, then micro-centroid pieces) within 1e-3"""
    keys, vals, rates, nk = _histo_stream(9)
    owners = ((np.arange(nk) + 1) % N).astype(np.uint32)
    rank, _ = deal(keys, N)

    def build(r, e):
        e.split_keys(2, np.arange(nk, dtype=np.uint32), owners)
        m = np.nonzero(rank == r)[0]
        for part in np.array_split(m, 2):
            e.ingest_split(histos=(keys[part], vals[part], rates[part]))

    out, _ = run_group(N, build, cap=(1, 1, 8, 1), exact_threshold=32768 if fast else 0)
    w = oracle.Worker(1, 1, nk, 1)
    w.histo(keys, vals, rates)
    wts = (np.float32(1.0) / rates).astype(np.float64)
    for k in range(nk):
        o = int(owners[k])
        f = out[o]
        i = f.histo_slot.tolist().index(k)
        ost = np.array(w.histo_stats(k))
        st = f.histo_stats[i]
        np.testing.assert_array_equal(st[[0, 1, 2, 5, 6, 7]], ost[[0, 1, 2, 5, 6, 7]])
        np.testing.assert_allclose(st[3:5], ost[3:5], rtol=1e-12)
        ref = [w.histo_quantile(k, p) for p in PCT]
        m = keys == k
        err = _rank_err(vals[m], wts[m], f.histo_quantiles[i], ref)
        assert err <= 1e-3, (k, err)
        if m.sum() <= 4096 or not fast:
            np.testing.assert_array_equal(f.histo_quantiles[i], ref)
        for r in range(N):
            if r != o:
                assert k not in out[r].histo_slot.tolist()


def test_rccl_group_of_one():
    """The RCCL transport itself, with one rank (a one-GPU box cannot hold two RCCL ranks):
    unique id, communicator, an all-reduce, and a flush that exchanges split keys over it."""
    uid = Comm.unique_id()
    c = Comm.rccl(uid, 1, 0, 0)
    try:
        assert (c.rank, c.nranks) == (0, 1)
        np.testing.assert_array_equal(c.allreduce_f64([1.5, -2.0], V._abi.VN_OP_MAX), [1.5, -2.0])
        with V.Engine((4, 1, 4, 4), percentiles=PCT, split_max_records=1 << 16) as e:
            e.set_comm(c)
            e.split_keys(0, np.array([1], np.uint32), np.array([0], np.uint32))
            e.split_keys(2, np.array([2], np.uint32), np.array([0], np.uint32))
            e.split_keys(3, np.array([3], np.uint32), np.array([0], np.uint32))
            e.ingest(counters=(np.array([1, 1], np.uint32), np.array([2.0, 3.0]), np.ones(2, np.float32)))
            v = np.arange(1.0, 6000.0)
            e.ingest_split(histos=(np.zeros(len(v), np.uint32), v, np.ones(len(v), np.float32)),
                           set_hashes=(np.zeros(3, np.uint32), np.array([5, 6, 7], np.uint64) << np.uint64(40)))
            f = e.flush()
        assert f.counter_value.tolist() == [5]
        w = oracle.Worker(1, 1, 1, 1)
        w.histo(np.zeros(len(v), np.uint32), v, np.ones(len(v), np.float32))
        assert f.histo_slot.tolist() == [2] and f.histo_stats[0][0] == len(v)
        ref = [w.histo_quantile(0, p) for p in PCT]
        assert _rank_err(v, np.ones(len(v)), f.histo_quantiles[0], ref) <= 1e-3
        assert f.set_slot.tolist() == [3] and f.set_estimate.tolist() == [3]
    finally:
        c.close()


@pytest.mark.parametrize("N", [1, 3])
def test_split_close_runs_combine_in_engine_thread(N):
    """vn_split_close: the split combine starts in the engine's own host thread; the result is the
    one vn_flush computes inline (sets bit-identical, histos within the rank bound)."""
    keys, vals, rates, nk = _histo_stream(4)
    owners = (np.arange(nk) % N).astype(np.uint32)
    rank, _ = deal(keys, N)
    rng = np.random.default_rng(8)
    skeys = rng.integers(0, 2, 300000).astype(np.uint32)
    shash = rng.integers(0, 2**63, 300000, dtype=np.uint64) * np.uint64(2)
    srank, _ = deal(skeys, N)
    sowners = np.array([0, (N - 1)], np.uint32)

    def build(r, e):
        e.split_keys(2, np.arange(nk, dtype=np.uint32), owners)
        e.split_keys(3, np.arange(2, dtype=np.uint32), sowners)
        m = np.nonzero(rank == r)[0]
        e.ingest_split(histos=(keys[m], vals[m], rates[m]))
        ms = np.nonzero(srank == r)[0]
        e.ingest_split(set_hashes=(skeys[ms], shash[ms]))

    outs = [run_group(N, build, cap=(1, 1, 8, 4), close=c)[0] for c in (False, True)]
    w = oracle.Worker(1, 1, nk, 1)
    w.histo(keys, vals, rates)
    for o in range(N):
        a, b = outs[0][o], outs[1][o]
        assert a.set_slot.tolist() == b.set_slot.tolist()
        assert a.set_estimate.tolist() == b.set_estimate.tolist()
        assert a.histo_slot.tolist() == b.histo_slot.tolist()
        np.testing.assert_array_equal(a.histo_stats[:, [0, 1, 2, 5, 6, 7]], b.histo_stats[:, [0, 1, 2, 5, 6, 7]])
        # the default (exact) mode: both are the single consumer's digests, bit for bit
        np.testing.assert_array_equal(a.histo_quantiles, b.histo_quantiles)
        for i, k in enumerate(a.histo_slot.tolist()):
            np.testing.assert_array_equal(a.histo_quantiles[i], [w.histo_quantile(k, p) for p in PCT])


def test_split_slot_with_direct_records_is_reported_not_mixed():
    """A split key's records belong to vn_ingest_split.  A window in which its slot also gets
    vn_ingest records (or imports) keeps the split combine's state -- moved on the engine's own
    stream after every ingest of the window -- and the flush reports the misuse once
    (warn_flags, a RuntimeWarning) while still returning the window: ADVICE r3, one misrouted
    record must not lose every other key's aggregates.  The next window is unaffected."""
    rng = np.random.default_rng(11)
    v = rng.lognormal(3.0, 1.0, 5000)
    comms = Comm.local(1)
    e = V.Engine((1, 1, 4, 4), percentiles=PCT, max_batch_records=1 << 16, split_max_records=1 << 16)
    try:
        e.set_comm(comms[0])
        e.split_keys(2, np.array([1], np.uint32), np.array([0], np.uint32))
        e.ingest_split(histos=(np.zeros(len(v), np.uint32), v, np.ones(len(v), np.float32)))
        e.ingest(histos=(np.array([1, 2], np.uint32), np.array([7.0, 8.0]), np.ones(2, np.float32)))
        with pytest.warns(RuntimeWarning, match="split key"):
            f0 = e.flush()
        assert f0.warn_flags & 16
        # the window survived: slot 2's own histogram, and slot 1 as the split combine left it
        assert f0.histo_slot.tolist() == [1, 2]
        assert f0.histo_stats[1][0] == 1.0 and f0.histo_stats[1][1] == 8.0
        w0 = oracle.Worker(1, 1, 1, 1)
        w0.histo(np.zeros(len(v), np.uint32), v, np.ones(len(v), np.float32))
        np.testing.assert_array_equal(f0.histo_quantiles[0], [w0.histo_quantile(0, p) for p in PCT])
        # the next window: split records only, no error, the single consumer's digest
        e.split_keys(2, np.array([1], np.uint32), np.array([0], np.uint32))
        e.ingest_split(histos=(np.zeros(len(v), np.uint32), v, np.ones(len(v), np.float32)))
        f = e.flush()
        assert f.histo_slot.tolist() == [1]
        w = oracle.Worker(1, 1, 1, 1)
        w.histo(np.zeros(len(v), np.uint32), v, np.ones(len(v), np.float32))
        np.testing.assert_array_equal(f.histo_quantiles[0], [w.histo_quantile(0, p) for p in PCT])
    finally:
        e.close()
        comms[0].close()
