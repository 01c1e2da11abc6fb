"""GPU parity at the BASELINE.json configs that are not the bench line.

C1  configs[0]: 1M timer samples over 1k keys into MergingDigest(100), p50/p99 flush.  Every
    key holds ~1000 samples (under the exact threshold), so the engine replays the reference's
    42-sample incremental merge and its quantiles must equal the restated Go bit for bit.
C2  configs[1]: HLL sets, 100k keys x 10M string members (Zipf 1.1, "m%010d" members from a
    5e7 universe), register-bit-exact against the restated clarkduvall/axiomhq sketch.
C5  configs[4]: a global veneur importing 1000 hosts' forwarded digests and sketches
    (worker.go:230-268): every key arrives from every host.  Scaled to 64 histogram keys and
    16 set keys per host so the oracle's per-payload Combine finishes in seconds; the
    per-key contribution counts (1000 payloads, 10^4..10^5 centroids per key) are the full
    config's.
"""
import numpy as np
import pytest

import oracle
import veneur_amd as V
from veneur_amd.dist import Group
from tests.util import PCT, engine_ingest, rank_errors, run_oracle
from tests.util import FAST_ONLY

pytestmark = pytest.mark.gpu


def _engine(n_slots, max_records, exact_threshold=0):
    return V.Engine(tuple(max(1, int(x)) for x in n_slots), percentiles=PCT, max_batch_records=max_records,
                    max_batch_member_bytes=max_records * 16, exact_threshold=exact_threshold)


def test_c1_single_worker_timers_bit_exact():
    d = V.synth(seed=0x5EED0001, n_keys=1000, zipf_s=0.0, mix=(0, 0, 1, 0), n_samples=1_000_000,
                rate_half=0.0, rate_tenth=0.0)
    n = d["n_slots"]
    assert n[2] == 1000 and len(d["h_slot"]) == 1_000_000
    w = run_oracle(d, n)
    with _engine(n, 1 << 20) as e:
        engine_ingest(e, d)
        f = e.flush()
    assert f.histo_slot.tolist() == list(range(1000))
    ost = np.array([w.histo_stats(int(s)) for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_stats[:, [0, 1, 2, 5, 6, 7]], ost[:, [0, 1, 2, 5, 6, 7]])
    for col in (3, 4):
        assert (np.abs(f.histo_stats[:, col] - ost[:, col]) / np.abs(ost[:, col])).max() <= 1e-12
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_quantiles, oq)  # p50/p90/p99/p99.9, every key


def test_c2_sets_100k_keys_10m_members_bit_exact():
    d = V.synth(seed=0x5EED0002, n_keys=100_000, zipf_s=1.1, mix=(0, 0, 0, 1), n_samples=10_000_000,
                member_universe=50_000_000)
    n = d["n_slots"]
    w = run_oracle(d, n)
    touched = [s for s in range(n[3]) if w.touched(3, s)]
    with _engine(n, 10_000_000) as e:
        engine_ingest(e, d)
        # full state (registers/b/nz or list/tmpSet) of every dense key and 2000 sparse ones
        dense = [s for s in touched if not w.set_sketch(s).sparse]
        rng = np.random.default_rng(2)
        sparse = [s for s in touched if w.set_sketch(s).sparse]
        probe = dense + [sparse[i] for i in rng.choice(len(sparse), 2000, replace=False)]
        for s in probe:
            st, sk = e.read_set(s), w.set_sketch(s)
            assert bool(st["sparse"]) == sk.sparse and st["b"] == sk.b, s
            if sk.sparse:
                assert np.array_equal(st["list"], sk.list_codes()), s
                assert np.array_equal(st["tmp"], sk.tmp_codes()), s
                assert st["list_bytes"] == sk.list_bytes(), s
            else:
                assert np.array_equal(st["registers"], sk.registers()), s
                assert st["nz"] == sk.nz, s
        f = e.flush()
    assert len(dense) > 50 and any(w.set_sketch(s).b > 0 for s in dense)  # dense + rebase exercised
    assert f.set_slot.tolist() == touched
    assert f.set_sparse.tolist() == [int(w.set_sketch(s).sparse) for s in touched]
    exp = np.array([w.set_estimate(s) for s in touched], np.uint64)
    bad = np.nonzero(f.set_estimate != exp)[0]
    assert len(bad) == 0, [(touched[i], int(f.set_estimate[i]), int(exp[i])) for i in bad[:10]]


def _c5_hosts(n_hosts, nh, ns, seed):
    """Each host is a local veneur: a Worker that Sample()s its own timers and set members,
    then forwards Histo.Export (GobEncode) and Set.Export (MarshalBinary) per key."""
    rng = np.random.default_rng(seed)
    for h in range(n_hosts):
        loc = oracle.Worker(1, 1, nh, ns)
        cnt = rng.integers(20, 200, nh)
        hs = np.repeat(np.arange(nh, dtype=np.uint32), cnt)
        hv = np.exp(rng.normal(3.9 + 0.01 * (h % 50), 1.0, len(hs)))
        hr = np.where(rng.random(len(hs)) < 0.1, np.float32(0.5), np.float32(1.0)).astype(np.float32)
        loc.histo(hs, hv, hr)
        # set sizes 1..20000 members: sparse payloads mostly, a few dense
        sc = np.minimum((rng.pareto(1.2, ns) * 200 + 1).astype(np.int64), 20000)
        ss = np.repeat(np.arange(ns, dtype=np.uint32), sc)
        sh = rng.integers(0, 2**63, len(ss), dtype=np.uint64) * np.uint64(2) + \
            rng.integers(0, 2, len(ss), dtype=np.uint64)
        loc.set_hashed(ss, sh)
        yield [loc.histo_gob(s) for s in range(nh)], [loc.set_sketch(s).marshal() for s in range(ns)]


@pytest.mark.parametrize("exact_threshold", [0, pytest.param(32768, marks=FAST_ONLY)])
def test_c5_global_import_1000_hosts(exact_threshold):
    """Default (exact) mode: every key re-Adds ~10^5 imported centroids, replayed merge by merge,
    so the quantiles are the reference's bit for bit; with the opt-in fast mode (threshold 32768)
    the keys take the geometric path and are held to 1e-3 rank error over the centroids."""
    n_hosts, nh, ns = 1000, 64, 16
    w = oracle.Worker(1, 1, nh, ns)
    cents = [[] for _ in range(nh)]
    hslots = np.arange(nh, dtype=np.uint32)
    sslots = np.arange(ns, dtype=np.uint32)
    with _engine((1, 1, nh, ns), 1 << 22, exact_threshold=exact_threshold) as e:
        for hp, sp in _c5_hosts(n_hosts, nh, ns, seed=5):
            e.import_histos(hslots, hp)
            e.import_sets(sslots, sp)
            for s, p in enumerate(hp):
                assert w.import_histo(s, p) == 0
                if exact_threshold:
                    t = oracle.MergingDigest(100.0)
                    t.gob_decode(p)
                    cents[s].append(t.centroids())
            for s, p in enumerate(sp):
                w.import_set(s, p)
        for s in range(ns):
            st, sk = e.read_set(s), w.set_sketch(s)
            assert bool(st["sparse"]) == sk.sparse and st["b"] == sk.b, s
            assert np.array_equal(st["registers"], sk.registers()), s
        f = e.flush()
    assert f.samples_imported == n_hosts * (nh + ns)
    assert f.set_estimate.tolist() == [w.set_estimate(s) for s in range(ns)]
    assert f.histo_slot.tolist() == list(range(nh))
    ost = np.array([w.histo_stats(s) for s in range(nh)])
    np.testing.assert_array_equal(f.histo_stats[:, [5, 6, 7]], ost[:, [5, 6, 7]])  # digest min/max/weight
    oq = np.array([[w.histo_quantile(s, p) for p in PCT] for s in range(nh)])
    if not exact_threshold:
        np.testing.assert_array_equal(f.histo_quantiles, oq)
        return
    stream = {"h_slot": np.concatenate([np.full(sum(len(m) for m, _ in cents[s]), s, np.uint32) for s in range(nh)]),
              "h_val": np.concatenate([m for s in range(nh) for m, _ in cents[s]]),
              "h_rate": np.concatenate([(1.0 / wt).astype(np.float32) for s in range(nh) for _, wt in cents[s]])}
    err = rank_errors(stream, f.histo_slot, f.histo_quantiles, oq)
    assert err.max() <= 1e-3, err.max()


def test_c5_bench_leg_small():
    """bench.py's C5 leg (hosts' payloads exported by a local engine, imported from HBM by a
    global engine) at a small scale: parity on every key."""
    from argparse import Namespace
    import bench
    r = bench.c5_leg(Namespace(seed=3, c5_histo_keys=300, c5_set_keys=60, c5_group=7, c5_hosts=40, c5_windows=1,
                               c5_parity_keys=300, c5_batch=1 << 20), 0, 1, Group(), 0)
    p = r["parity"]
    assert p["keys_checked"] == {"histo": 300, "set": 60}
    assert p["histo_weight_min_max_exact"] and p["set_estimates_exact"]
    assert p["histo_quantiles_bit_exact"] and p["histo_rank_error_max"] == 0.0, p
    assert r["payloads_per_window"] == 40 * 360 and r["imports_per_s"] > 0


def test_c5_bench_leg_sharded_over_two_ranks():
    """the C5 leg as rank 0 and rank 1 of N = 2 (run one after the other on this GPU): each rank
    keeps its keys' payloads (digest % 2), the two shares cover every key once, and each rank's
    imports are bit-exact against the oracle on every key it owns"""
    from argparse import Namespace
    import bench
    keys = [0, 0]
    for r in range(2):
        res = bench.c5_leg(Namespace(seed=5, c5_histo_keys=120, c5_set_keys=30, c5_group=8, c5_hosts=24,
                                     c5_windows=1, c5_parity_keys=300, c5_batch=1 << 20), r, 2, Group(), 0)
        p = res["parity"]
        assert p["histo_weight_min_max_exact"] and p["set_estimates_exact"] and p["histo_quantiles_bit_exact"], p
        hk, sk = res["ranks"]["histo_set_keys"][0]
        assert p["keys_checked"] == {"histo": hk, "set": sk} and hk > 0 and sk > 0
        keys[0] += hk
        keys[1] += sk
    assert keys == [120, 30]


def test_c5_import_sliced_by_centroids():
    """one vn_import_histos_device call whose centroids exceed max_batch_records: the engine cuts
    it into payload slices (k_import_slices) and drains each in arrival order -- the quantiles
    are those of importing the payloads one call after another (bit-exact vs the oracle)"""
    from argparse import Namespace
    import bench
    r = bench.c5_leg(Namespace(seed=4, c5_histo_keys=64, c5_set_keys=8, c5_group=16, c5_hosts=64, c5_windows=2,
                               c5_parity_keys=64, c5_batch=60_000), 0, 1, Group(), 0)
    p = r["parity"]
    assert p["histo_weight_min_max_exact"] and p["set_estimates_exact"] and p["histo_quantiles_bit_exact"], p
