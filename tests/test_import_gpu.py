"""GPU parity of Worker.ImportMetric for histograms and sets (worker.go:230-268).

The payloads are what a global veneur receives from locals: GobEncode()d MergingDigests
(merging_digest.go:361-380) and MarshalBinary()d axiomhq sketches (hyperloglog.go:270-315),
produced here by the oracle (whose gob encoder reproduces fixtures/import.uncompressed byte for
byte, tests/test_oracle_kats.py).  The engine decodes and merges them on the GPU; the oracle's
Worker.import_histo / import_set (Histo.Combine / Set.Combine restated) is the checker.
MergingDigest.Merge re-Adds the other digest's centroids in rand.Perm order (time-seeded in the
reference); the engine Adds them in stored order, and the oracle is given that permutation.
"""
import os

import numpy as np
import pytest

import oracle
import veneur_amd as V
from tests.util import PCT, run_oracle
from tests.util import FAST_ONLY

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def make_engine(n_slots, pct=PCT, max_records=1 << 18, exact_threshold=0):
    return V.Engine(tuple(max(1, x) for x in n_slots), percentiles=pct, max_batch_records=max_records,
                    max_batch_member_bytes=max_records * 16, exact_threshold=exact_threshold)


def identity(n):
    return np.arange(n, dtype=np.int64)


def digest_payload(rng, n_samples, mu=3.9, rate_tenth=0.0):
    """A local veneur's forwarded digest: n samples Add()ed, then GobEncode (Histo.Export)."""
    td = oracle.MergingDigest(100.0)
    v = np.exp(rng.normal(mu, 1.0, n_samples))
    w = np.where(rng.random(n_samples) < rate_tenth, 10.0, 1.0)
    td.add_many(v, w)
    return td.gob_encode()


def test_import_histo_fixture_digest():
    """fixtures/import.uncompressed: one digest of {1,2,7,8,100} forwarded to a global."""
    gob = open(os.path.join(GOLD, "tdigest_1_2_7_8_100.gob"), "rb").read()
    with make_engine((1, 1, 1, 1), pct=(0.5, 0.75, 0.99)) as e:
        e.import_histos([0], [gob])
        m, w, st = e.read_histo(0)
        # Merge Add()ed the 5 centroids as pending temps; Local* stats untouched
        assert st[0] == 0 and st[1] == np.inf and st[2] == -np.inf and st[5] == 1 and st[6] == 100
        f = e.flush()
    assert f.samples_imported == 1 and f.samples_processed == 0
    assert f.histo_quantiles[0][0] == 6 and f.histo_quantiles[0][1] == 42.375
    assert f.histo_quantiles[0][2] == pytest.approx(97.7, rel=1e-15)


def _check_histos(e, w, slots, exact=True):
    f = e.flush()
    exp = np.array([s for s in slots if w.touched(2, int(s))], np.uint32)
    assert np.array_equal(f.histo_slot, exp)
    ost = np.array([w.histo_stats(int(s)) for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_stats[:, [0, 1, 2, 5, 6, 7]], ost[:, [0, 1, 2, 5, 6, 7]])
    for col in (3, 4):
        rel = np.abs(f.histo_stats[:, col] - ost[:, col]) / np.maximum(np.abs(ost[:, col]), 1e-300)
        assert rel.max() <= 1e-12
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    if exact:
        np.testing.assert_array_equal(f.histo_quantiles, oq)
    return f, oq


def test_import_histos_many_hosts_bit_exact():
    """64 keys x 40 hosts' digests (integer weights), interleaved with local samples: every
    key stays under the exact threshold, so quantiles match the restated Go bit for bit."""
    rng = np.random.default_rng(11)
    nk, hosts = 64, 40
    w = oracle.Worker(1, 1, nk, 1)
    with make_engine((1, 1, nk, 1)) as e:
        for h in range(hosts):
            slots = rng.permutation(nk)[: rng.integers(nk // 2, nk)].astype(np.uint32)
            pays = [digest_payload(rng, int(rng.integers(1, 300)), rate_tenth=0.1) for _ in slots]
            e.import_histos(slots, pays)
            for s, p in zip(slots, pays):
                t = oracle.MergingDigest(100.0)
                t.gob_decode(p)
                assert w.import_histo(int(s), p, identity(len(t.centroids()[0]))) == 0
            if h % 7 == 3:  # local samples of the same keys between imports (ProcessMetric)
                ls = rng.integers(0, nk, 500).astype(np.uint32)
                lv = np.exp(rng.normal(3.0, 1.0, 500))
                lr = np.where(rng.random(500) < 0.2, np.float32(0.5), np.float32(1.0)).astype(np.float32)
                e.ingest(histos=(ls, lv, lr))
                w.histo(ls, lv, lr)
        _check_histos(e, w, range(nk))


@FAST_ONLY
def test_import_histos_hot_key_rank_error():
    """One key imports far more centroids than the exact threshold: the hot-key batch merge
    applies the remainder; quantiles within 1e-3 rank error of the restated Go."""
    rng = np.random.default_rng(12)
    w = oracle.Worker(1, 1, 2, 1)
    allv = []
    with make_engine((1, 1, 2, 1), max_records=1 << 20, exact_threshold=4096) as e:
        for h in range(8):
            pays, slots = [], []
            for _ in range(200):
                td = oracle.MergingDigest(100.0)
                v = np.exp(rng.normal(3.9, 1.0, 50))
                td.add_many(v, np.ones(50))
                allv.append(v)
                pays.append(td.gob_encode())
                slots.append(0)
            e.import_histos(np.array(slots, np.uint32), pays)
            for p in pays:
                t = oracle.MergingDigest(100.0)
                t.gob_decode(p)
                w.import_histo(0, p, identity(len(t.centroids()[0])))
        f = e.flush()
    oq = np.array([w.histo_quantile(0, p) for p in PCT])
    vals = np.sort(np.concatenate(allv))
    F = lambda q: np.searchsorted(vals, q, side="right") / len(vals)
    err = max(abs(F(a) - F(b)) for a, b in zip(f.histo_quantiles[0], oq))
    assert err <= 1e-3, err
    assert f.histo_stats[0][5] == w.histo_stats(0)[5] and f.histo_stats[0][6] == w.histo_stats(0)[6]


def test_import_histos_sliced_through_a_small_run_bit_exact():
    """a call holding far more centroids than the import run (max_batch_records 256)
    is cut into slices of whole payloads, each at most the run -- payloads of 50-250 samples
    (up to ~130 centroids) can no longer make a slice of up to 1.5x the run -- and merged in
    arrival order: bit-exact against the restated Go's per-payload Merge."""
    rng = np.random.default_rng(23)
    nk, npay = 6, 180
    w = oracle.Worker(1, 1, nk, 1)
    slots = rng.integers(0, nk, npay).astype(np.uint32)
    pays = [digest_payload(rng, int(rng.integers(50, 250)), rate_tenth=0.1) for _ in slots]
    for s, p in zip(slots, pays):
        t = oracle.MergingDigest(100.0)
        t.gob_decode(p)
        assert w.import_histo(int(s), p, identity(len(t.centroids()[0]))) == 0
    with make_engine((1, 1, nk, 1), max_records=256) as e:
        e.import_histos(slots, pays)
        _check_histos(e, w, range(nk))


def test_import_histos_more_slices_than_one_cut_pass_bit_exact():
    """A call cut into more slices than one device pass of k_import_cuts finds (1024): the histo
    class capped at 64 records, so each slice holds one or two 20-40-sample digests; 1300 payloads,
    merged in arrival order, bit-exact against the restated Go's per-payload Merge."""
    rng = np.random.default_rng(29)
    nk, npay = 5, 1300
    w = oracle.Worker(1, 1, nk, 1)
    slots = rng.integers(0, nk, npay).astype(np.uint32)
    pays = [digest_payload(rng, int(rng.integers(20, 40))) for _ in slots]
    for s, p in zip(slots, pays):
        t = oracle.MergingDigest(100.0)
        t.gob_decode(p)
        assert w.import_histo(int(s), p, identity(len(t.centroids()[0]))) == 0
    with V.Engine((1, 1, nk, 1), percentiles=PCT, max_batch_records=1 << 14, max_batch_member_bytes=1 << 18,
                  max_class_records=(0, 0, 64, 0)) as e:
        e.import_histos(slots, pays)
        _check_histos(e, w, range(nk))


def test_import_histos_empty_digests_among_others_bit_exact():
    """Digests without centroids (a local veneur's key that received nothing) mixed into a call,
    some keys receiving only those: the drain's key segments come from the payload table, where an
    empty digest is a payload with no records -- every key's state, and which keys flush, as the
    restated Go's per-payload Merge."""
    rng = np.random.default_rng(31)
    nk, npay = 8, 300
    w = oracle.Worker(1, 1, nk, 1)
    slots = rng.integers(0, nk, npay).astype(np.uint32)
    slots[rng.random(npay) < 0.1] = nk - 1  # key nk-1: empty digests only
    pays = []
    for s in slots:
        empty = s == nk - 1 or rng.random() < 0.25
        pays.append(digest_payload(rng, 0 if empty else int(rng.integers(5, 120))))
    for s, p in zip(slots, pays):
        t = oracle.MergingDigest(100.0)
        t.gob_decode(p)
        assert w.import_histo(int(s), p, identity(len(t.centroids()[0]))) == 0
    with V.Engine((1, 1, nk, 1), percentiles=PCT, max_batch_records=1 << 14, max_batch_member_bytes=1 << 18,
                  max_class_records=(0, 0, 512, 0)) as e:  # (a run of 512 centroids: several drains)
        e.import_histos(slots, pays)
        _check_histos(e, w, range(nk))


def test_import_histos_oversize_digest_refused_before_anything_applies():
    """a payload larger than the run is refused up front: nothing of the call is applied"""
    rng = np.random.default_rng(24)
    small = digest_payload(rng, 30)
    big = digest_payload(rng, 400)  # > 64 centroids
    with make_engine((1, 1, 4, 1), max_records=64) as e:
        with pytest.raises(V.EngineError):
            e.import_histos([0, 1, 2], [small, small, big])
        e.import_histos([3], [small])
        f = e.flush()
    assert f.histo_slot.tolist() == [3]


def test_import_histos_malformed_fails_loudly():
    good = digest_payload(np.random.default_rng(1), 20)
    with make_engine((1, 1, 4, 1)) as e:
        with pytest.raises(V.EngineError, match="rc=-4"):
            e.import_histos([0, 1], [good, good[:-3]])
        with pytest.raises(V.EngineError, match="rc=-4"):
            e.import_histos([0], [b"\x00\x01\x02"])
        # nothing was applied; the engine keeps working
        e.import_histos([2], [good])
        f = e.flush()
    assert f.histo_slot.tolist() == [2]


# ------------------------------------------------------------------ sets
def random_hashes(rng, n):
    return rng.integers(0, 2**63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)


def sketch_payload(rng, n, p=14):
    """A local veneur's forwarded set: n random members inserted, then MarshalBinary."""
    sk = oracle.Sketch(p)
    for h in random_hashes(rng, n):
        sk.insert_hash(int(h))
    return sk.marshal()


def _set_state_equal(e, w, slot):
    st = e.read_set(slot)
    sk = w.set_sketch(slot)
    assert bool(st["sparse"]) == sk.sparse, slot
    assert st["b"] == sk.b, slot
    if sk.sparse:
        assert np.array_equal(st["list"], sk.list_codes()), slot
        assert np.array_equal(st["tmp"], sk.tmp_codes()), slot
        assert st["list_bytes"] == sk.list_bytes(), slot
    else:
        assert np.array_equal(st["registers"], sk.registers()), slot
        assert st["nz"] == sk.nz, slot


def test_import_sets_every_merge_path_bit_exact():
    """sparse<-sparse (with and without the mergeSparse trigger and the toNormal switch),
    sparse<-dense, dense<-sparse, dense<-dense with either base higher, a precision-16 payload
    (skipped, key still Upserted), keys that already hold local samples; state and Estimate
    bit-exact against the restated axiomhq Merge."""
    rng = np.random.default_rng(21)
    nk = 12
    small = [sketch_payload(rng, k) for k in (1, 30, 150)]
    mid = [sketch_payload(rng, k) for k in (400, 3000)]
    big = [sketch_payload(rng, k) for k in (9000, 40000)]
    reb = sketch_payload(rng, 400_000)
    p16 = sketch_payload(rng, 100, p=16)
    tmp = oracle.Sketch()
    tmp.unmarshal(reb)
    assert not tmp.sparse and tmp.b > 0  # a based (rebased) dense payload
    w = oracle.Worker(1, 1, 1, nk)
    # local samples first: keys 4,5 sparse, 6,7 dense, 8 dense with b > 0
    loc_slots, loc_h = [], []
    for s, n in ((4, 200), (5, 200), (6, 20000), (7, 20000), (8, 400_000)):
        loc_slots.append(np.full(n, s, np.uint32))
        loc_h.append(random_hashes(rng, n))
    ls, lh = np.concatenate(loc_slots), np.concatenate(loc_h)
    w.set_hashed(ls, lh)
    calls = [
        ([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11],
         [small[0], small[1], mid[0], big[0], small[2], mid[1], small[1], big[1], reb, p16, reb, mid[1]]),
        ([0, 0, 1, 2, 3, 9, 10, 11, 11, 8, 6], [small[1], mid[1], big[0], reb, small[0], small[2], big[1], small[0],
                                                 big[0], big[1], mid[0]]),
        ([0, 0, 0, 0, 0, 2, 5], [mid[0], mid[1], small[2], small[1], small[0], mid[0], reb]),
    ]
    with make_engine((1, 1, 1, nk), max_records=1 << 19) as e:
        e.ingest(set_hashes=(ls, lh))
        for slots, pays in calls:
            e.import_sets(np.array(slots, np.uint32), pays)
            for s, p in zip(slots, pays):
                w.import_set(s, p)
        for s in range(nk):
            _set_state_equal(e, w, s)
        f = e.flush()
    assert f.set_slot.tolist() == list(range(nk))
    assert f.samples_imported == sum(len(c[0]) for c in calls)
    exp = [w.set_estimate(s) for s in range(nk)]
    assert f.set_estimate.tolist() == exp


def test_import_sets_many_hosts_sparse_trigger_path():
    """200 keys x 30 hosts' small sparse sketches: the tmpSet/list union and the 164-code
    trigger across many payloads per key."""
    rng = np.random.default_rng(22)
    nk, hosts = 200, 30
    pays = [sketch_payload(rng, int(n)) for n in rng.integers(1, 120, 64)]
    w = oracle.Worker(1, 1, 1, nk)
    with make_engine((1, 1, 1, nk)) as e:
        for h in range(hosts):
            slots = rng.integers(0, nk, 150).astype(np.uint32)
            pl = [pays[i] for i in rng.integers(0, len(pays), len(slots))]
            e.import_sets(slots, pl)
            for s, p in zip(slots, pl):
                w.import_set(int(s), p)
        touched = [s for s in range(nk) if w.touched(3, s)]
        for s in touched:
            _set_state_equal(e, w, s)
        f = e.flush()
    assert f.set_estimate.tolist() == [w.set_estimate(s) for s in touched]


def overflow_payload(rng, n, n_over):
    """A sparse sketch holding n random members plus n_over members whose rho is 50 (hash bits
    below the register index all zero): overflow codes for any base below 35."""
    sk = oracle.Sketch(14)
    for h in random_hashes(rng, n):
        sk.insert_hash(int(h))
    for i in rng.integers(0, 1 << 14, n_over):
        sk.insert_hash((int(i) << 50) | 1)
    return sk.marshal()


def test_import_sets_dense_keys_many_sparse_payloads_bit_exact():
    """Dense keys (fresh, nearly full, rebased b > 0) receiving hundreds of sparse payloads of
    Lomax sizes in one call -- the run of plain register maxes, a wave per payload --
    mixed with payloads carrying overflow codes, dense payloads and skipped precisions, so the
    runs are cut where a rebase may happen; registers, b, nz and estimates bit-exact."""
    rng = np.random.default_rng(24)
    nk = 6
    w = oracle.Worker(1, 1, 1, nk)
    loc_slots, loc_h = [], []
    for s, n in ((0, 20000), (1, 60000), (2, 400_000), (3, 150_000), (5, 9000)):
        loc_slots.append(np.full(n, s, np.uint32))
        loc_h.append(random_hashes(rng, n))
    ls, lh = np.concatenate(loc_slots), np.concatenate(loc_h)
    w.set_hashed(ls, lh)
    sizes = np.minimum((rng.pareto(1.2, 400) * 50).astype(int) + 1, 6000)
    pool = [sketch_payload(rng, int(n)) for n in sizes[:360]]
    pool += [overflow_payload(rng, int(n), int(k)) for n, k in zip(sizes[360:], rng.integers(1, 4, 40))]
    pool += [sketch_payload(rng, 12000), sketch_payload(rng, 100, p=16)]
    with make_engine((1, 1, 1, nk), max_records=1 << 20) as e:
        e.ingest(set_hashes=(ls, lh))
        for call in range(3):
            slots = rng.integers(0, nk, 700).astype(np.uint32)
            idx = rng.integers(0, len(pool), len(slots))
            idx[rng.random(len(slots)) < 0.01] = len(pool) - 2  # a few dense payloads
            pl = [pool[i] for i in idx]
            e.import_sets(slots, pl)
            for s, p in zip(slots, pl):
                w.import_set(int(s), p)
            for s in range(nk):
                if w.touched(3, s):
                    _set_state_equal(e, w, s)
        assert w.set_sketch(3).b > 0 and w.set_sketch(4).b == 0  # a rebase inside the imports
        f = e.flush()
    assert f.set_estimate.tolist() == [w.set_estimate(s) for s in range(nk) if w.touched(3, s)]


def test_import_sets_malformed_fails_loudly():
    rng = np.random.default_rng(23)
    good = sketch_payload(rng, 50)
    with make_engine((1, 1, 1, 4)) as e:
        with pytest.raises(V.EngineError, match="rc=-4"):
            e.import_sets([0, 1], [good, good[:-2]])
        e.import_sets([2], [good])
        f = e.flush()
    assert f.set_slot.tolist() == [2]


# ------------------------------------------------------------------ export (forward encoders)
def test_export_histos_byte_identical_and_roundtrip():
    """Histo.Export = GobEncode (merging_digest.go:361-380): the engine's bytes equal the
    restated Go encoder's (which reproduces fixtures/import.uncompressed), and a global that
    imports them holds the local's digest."""
    d = V.synth(seed=61, n_keys=80, zipf_s=1.0, mix=(0, 0, 1, 0), n_samples=30_000)
    w = run_oracle(d, d["n_slots"])
    slots = np.array([s for s in range(d["n_slots"][2]) if w.touched(2, s)], np.uint32)
    with make_engine(d["n_slots"]) as e:
        e.ingest(histos=(d["h_slot"], d["h_val"], d["h_rate"]))
        pays = e.export_histos(slots)
        again = e.export_histos(slots[::-1])  # pending temps merged once; repeats are stable
    exp = [w.histo_gob(int(s)) for s in slots]
    assert pays == exp
    assert again == exp[::-1]
    with make_engine(d["n_slots"]) as g:  # the global
        g.import_histos(slots, pays)
        f = g.flush()
    w2 = oracle.Worker(*d["n_slots"])
    for s, p in zip(slots, pays):
        t = oracle.MergingDigest(100.0)
        t.gob_decode(p)
        w2.import_histo(int(s), p, identity(len(t.centroids()[0])))
    oq = np.array([[w2.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_quantiles, oq)


def test_export_sets_byte_identical_and_roundtrip():
    """Set.Export = MarshalBinary (hyperloglog.go:270-315), sparse and dense (b > 0 too)."""
    rng = np.random.default_rng(62)
    sizes = [0, 1, 50, 163, 164, 900, 6000, 30000, 400_000]
    slots = np.concatenate([np.full(n, i, np.uint32) for i, n in enumerate(sizes)])
    hashes = random_hashes(rng, len(slots))
    perm = rng.permutation(len(slots))
    slots, hashes = slots[perm], hashes[perm]
    nk = len(sizes)
    w = oracle.Worker(1, 1, 1, nk)
    w.set_hashed(slots, hashes)
    with make_engine((1, 1, 1, nk), max_records=1 << 19) as e:
        e.ingest(set_hashes=(slots, hashes))
        touched = [s for s in range(nk) if w.touched(3, s)]
        pays = e.export_sets(touched)
    exp = [w.set_sketch(s).marshal() for s in touched]
    assert pays == exp
    with make_engine((1, 1, 1, nk), max_records=1 << 19) as g:
        g.import_sets(touched, pays)
        f = g.flush()
    assert f.set_estimate.tolist() == [w.set_estimate(s) for s in touched]
