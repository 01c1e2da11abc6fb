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
from tests.util import PCT

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
