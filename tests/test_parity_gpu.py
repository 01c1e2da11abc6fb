"""Parity of the HIP engine (through the C-ABI) with the CPU oracle on identical inputs.

Bars (north_star): HLL registers / estimates and integer counters bit-exact; float sums
within 1e-12 relative; t-digest quantiles within 1e-3 rank error.  Each case names the
reference test or semantics it checks.
"""
import struct

import numpy as np
import pytest

import oracle
from tests.util import PCT, engine_ingest, rank_errors, run_oracle, split_batches

pytestmark = pytest.mark.gpu

import veneur_amd as V  # noqa: E402  (fails loudly when the HIP library is missing)
from tests.util import FAST_ONLY


def make_engine(n_slots, compression=100.0, pct=PCT, max_records=1 << 20, exact_threshold=0):
    caps = tuple(max(1, int(n)) for n in n_slots)
    return V.Engine(caps, compression=compression, percentiles=pct, max_batch_records=max_records,
                    max_batch_member_bytes=max_records * 24, exact_threshold=exact_threshold)


# ------------------------------------------------------------------ metro64 / HLL encoding
def test_metro64_kat_on_device():  # go-metro metro_test.go:9-27
    key63 = b"012345678901234567890123456789012345678901234567890123456789012"
    out = V.metro64_device([key63, key63], seed=0)
    assert int(out[0]) == struct.unpack("<Q", bytes([0x6B, 0x75, 0x3D, 0xAE, 0x06, 0x70, 0x4B, 0xAD]))[0]
    out1 = V.metro64_device([key63], seed=1)
    assert int(out1[0]) == struct.unpack("<Q", bytes([0x3B, 0x0D, 0x48, 0x1C, 0xF4, 0xB9, 0xB8, 0xDF]))[0]


def test_metro64_all_lengths_vs_oracle():
    rng = np.random.default_rng(0)
    members = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in list(range(0, 80)) * 3 + [200, 1000, 4097]]
    got = V.metro64_device(members, seed=1337)
    for m, g in zip(members, got):
        assert int(g) == oracle.metro64(m, 1337)


# ------------------------------------------------------------------ counters / gauges
def test_counter_kats():  # samplers_test.go:46-106
    with make_engine((4, 1, 1, 1)) as e:
        e.ingest(counters=([0, 1, 2], [1.0, 5.0, 5.0], [1.0, 1.0, 0.5]))
        e.import_counters([3], [10])
        e.import_counters([3], [28])
        f = e.flush()
        assert dict(zip(f.counter_slot.tolist(), f.counter_value.tolist())) == {0: 1, 1: 5, 2: 10, 3: 38}


def test_counter_go_conversion_edges():  # samplers.go:133 float32 1/rate, int64 truncation, wrap
    slots = [0, 1, 2, 3, 3]
    vals = [3.7, -2.9, 1e300, 9.2e18, 9.2e18]
    rates = np.array([0.3, 0.1, 1.0, 0.5, 0.5], np.float32)
    w = oracle.Worker(4, 0, 0, 0)
    w.counter(slots, vals, rates)
    with make_engine((4, 1, 1, 1)) as e:
        e.ingest(counters=(slots, vals, rates))
        f = e.flush()
        got = dict(zip(f.counter_slot.tolist(), f.counter_value.tolist()))
    assert got == {s: w.counter_value(s) for s in range(4)}


def test_gauge_last_write_wins_across_batches_and_imports():  # samplers.go:198-249
    rng = np.random.default_rng(1)
    n_slots = 50
    batches = [(rng.integers(0, n_slots, 5000).astype(np.uint32), rng.random(5000) * 1000) for _ in range(3)]
    w = oracle.Worker(0, n_slots, 0, 0)
    with make_engine((1, n_slots, 1, 1)) as e:
        for s, v in batches:
            e.ingest(gauges=(s, v))
            w.gauge(s, v)
        e.import_gauges([7, 7, 8], [1.5, 2.5, 3.5])
        for s, v in zip([7, 7, 8], [1.5, 2.5, 3.5]):
            w.import_gauge(s, v)
        f = e.flush()
    exp = {s: w.gauge_value(s) for s in range(n_slots) if w.touched(1, s)}
    assert dict(zip(f.gauge_slot.tolist(), f.gauge_value.tolist())) == exp


# ------------------------------------------------------------------ histos
def test_histo_kat():  # samplers_test.go:192-283 (+ HistoSampleRate 354-382)
    with make_engine((1, 1, 2, 1), pct=(0.5, 0.9)) as e:
        e.ingest(histos=([0] * 5 + [1] * 5, [5, 10, 15, 20, 25] * 2, [1.0] * 5 + [0.5] * 5))
        f = e.flush()
    st, q = f.histo_stats[0], f.histo_quantiles[0]
    assert (st[2], st[1], st[3], st[0]) == (25, 5, 75, 5)
    assert st[3] / st[0] == 15
    assert st[0] / st[4] == 5.0 / ((1.0 / 5) + (1.0 / 10) + (1.0 / 15) + (1.0 / 20) + (1.0 / 25))
    assert q[0] == 15 and q[1] == 23.75
    assert f.histo_stats[1][2] == 25 and f.histo_stats[1][0] == 10


def test_histo_import_fixture_digest_quantiles():
    """Centroids of fixtures/import.uncompressed ({1,2,7,8,100}) as samples -> 6 / 42.375 / 97.7."""
    with make_engine((1, 1, 1, 1), pct=(0.5, 0.75, 0.99)) as e:
        e.ingest(histos=([0] * 5, [1.0, 2.0, 7.0, 8.0, 100.0], [1.0] * 5))
        m, w, st = e.read_histo(0)
        # as in the reference the 5 samples are still pending temps (Add never filled 42);
        # Quantile merges them: digest min/max are already tracked by Add
        assert len(m) == 0 and st[5] == 1 and st[6] == 100 and st[0] == 5
        f = e.flush()
    assert f.histo_quantiles[0][0] == 6 and f.histo_quantiles[0][1] == 42.375
    assert f.histo_quantiles[0][2] == pytest.approx(97.7, rel=1e-15)


def _histo_parity(stream, n_slots, batches=1, compression=100.0, max_rank=1e-3, exact_threshold=0):
    w = run_oracle(stream, n_slots)
    counts = np.bincount(stream["h_slot"], minlength=n_slots[2])
    thr = exact_threshold if exact_threshold and exact_threshold < 0xFFFFFFFF else 1 << 62  # 0: exact
    with make_engine(n_slots, compression=compression, max_records=max(1 << 16, len(stream["h_slot"])),
                     exact_threshold=exact_threshold) as e:
        for d in split_batches(stream, batches):
            engine_ingest(e, d)
        f = e.flush()
    slots = f.histo_slot
    exp_slots = np.array([s for s in range(n_slots[2]) if w.touched(2, s)], np.uint32)
    assert np.array_equal(slots, exp_slots)
    ost = np.array([w.histo_stats(int(s)) for s in slots])
    # min / max bit-exact (math.Min / math.Max), weights exact (integer weights)
    assert np.array_equal(f.histo_stats[:, 1], ost[:, 1])
    assert np.array_equal(f.histo_stats[:, 2], ost[:, 2])
    assert np.array_equal(f.histo_stats[:, 0], ost[:, 0])
    assert np.array_equal(f.histo_stats[:, 7], ost[:, 7])
    # float sums within 1e-12 relative
    for col in (3, 4):
        rel = np.abs(f.histo_stats[:, col] - ost[:, col]) / np.abs(ost[:, col])
        assert rel.max() <= 1e-12, (col, rel.max())
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in slots])
    # keys under the exact threshold replay MergingDigest.Add bit-for-bit: identical quantiles
    exact = counts[slots] <= thr
    if exact.any():
        bad = np.nonzero(np.any(f.histo_quantiles[exact] != oq[exact], axis=1))[0]
        assert len(bad) == 0, [(int(slots[exact][i]), f.histo_quantiles[exact][i], oq[exact][i]) for i in bad[:5]]
    errs = rank_errors(stream, slots, f.histo_quantiles, oq)
    assert errs.max() <= max_rank, errs.max(axis=0)
    return errs


def test_histo_random_parity_single_batch():
    d = V.synth(seed=21, n_keys=400, zipf_s=1.0, mix=(0, 0, 1, 0), n_samples=200_000)
    _histo_parity(d, d["n_slots"])


def test_histo_random_parity_multi_batch():
    d = V.synth(seed=22, n_keys=300, zipf_s=1.1, mix=(0, 0, 1, 0), n_samples=150_000)
    _histo_parity(d, d["n_slots"], batches=4)


@FAST_ONLY
def test_histo_hot_key_multi_chunk():
    """keys with far more samples than the exact threshold: batch merge of the hot remainder
    (multi-chunk chain path) after an exact prefix; rank-error parity."""
    d = V.synth(seed=23, n_keys=20, zipf_s=2.0, mix=(0, 0, 1, 0), n_samples=600_000)
    _histo_parity(d, d["n_slots"], batches=2, exact_threshold=20000)


def test_histo_exact_replay_all_keys_multi_batch():
    """threshold above every key: bit-identical quantiles across 5 ingest batches"""
    d = V.synth(seed=24, n_keys=200, zipf_s=1.0, mix=(0, 0, 1, 0), n_samples=100_000)
    _histo_parity(d, d["n_slots"], batches=5, exact_threshold=0xFFFFFFFF)


def test_histo_compression_1000_accuracy():  # histo_test.go:11-25 (delta=1000)
    rng = np.random.default_rng(5)
    vals = rng.random(200_000)
    with make_engine((1, 1, 1, 1), compression=1000.0, pct=(0.5,), max_records=1 << 18) as e:
        e.ingest(histos=(np.zeros(len(vals), np.uint32), vals, np.ones(len(vals), np.float32)))
        m, w, st = e.read_histo(0)
        f = e.flush()
    assert f.histo_quantiles[0][0] == pytest.approx(0.5, rel=0.02)
    # the main centroids hold every merged sample; the rest are still pending temps (178 at
    # delta 1000), as in the reference
    assert w.sum() == st[7] and 0 < len(vals) - w.sum() <= 178 and f.histo_stats[0][0] == len(vals)
    assert st[5] >= 0 and st[6] < 1
    t = oracle.MergingDigest(1000.0)
    t.add_many(vals, np.ones(len(vals)))
    assert f.histo_quantiles[0][0] == t.quantile(0.5)


def test_histo_signed_zero_and_negative():  # math.Min(-0, +0) = -0
    vals = [0.0, -0.0, -5.0, 3.0, -0.0, 0.0]
    w = oracle.Worker(0, 0, 1, 0)
    w.histo([0] * 6, vals, [1.0] * 6)
    with make_engine((1, 1, 1, 1)) as e:
        e.ingest(histos=([0] * 6, vals, [1.0] * 6))
        f = e.flush()
    ost = w.histo_stats(0)
    assert f.histo_stats[0][1] == ost[1] == -5.0
    assert np.signbit(f.histo_stats[0][2]) == np.signbit(ost[2])


# ------------------------------------------------------------------ sets (HLL)
def test_set_kat():  # samplers_test.go:144-168
    members = [b"5", b"5", b"123", b"2147483647", b"-2147483648"]
    off = np.cumsum([0] + [len(m) for m in members]).astype(np.uint32)
    with make_engine((1, 1, 1, 1)) as e:
        e.ingest(sets=(np.zeros(5, np.uint32), off, np.frombuffer(b"".join(members), np.uint8)))
        f = e.flush()
    assert f.set_estimate.tolist() == [4]


def test_set_nophash_cardinality_kat():  # hyperloglog_test.go:175-208 (p=14 here; sparse path)
    hashes = [0x00010FFFFFFFFFFF, 0x00020FFFFFFFFFFF, 0x00030FFFFFFFFFFF, 0x00040FFFFFFFFFFF, 0x00050FFFFFFFFFFF,
              0x00050FFFFFFFFFFF]
    with make_engine((1, 1, 1, 1)) as e:
        e.ingest(set_hashes=(np.zeros(6, np.uint32), np.array(hashes, np.uint64)))
        f = e.flush()
    assert f.set_estimate.tolist() == [5]


def _set_state_equal(e, w, slot):
    st = e.read_set(slot)
    sk = w.set_sketch(slot)
    assert bool(st["sparse"]) == sk.sparse, slot
    assert st["b"] == sk.b, slot
    if sk.sparse:
        assert np.array_equal(st["list"], sk.list_codes()), slot
        assert np.array_equal(st["tmp"], sk.tmp_codes()), slot
        assert st["list_bytes"] == sk.list_bytes()
    else:
        assert np.array_equal(st["registers"], sk.registers()), slot
        assert st["nz"] == sk.nz, slot


def _set_parity(stream, n_slots, batches=1, hashed=False, check_state=True):
    w = run_oracle(stream, n_slots, hashed=hashed)
    with make_engine(n_slots, max_records=max(1 << 16, len(stream["s_slot"]))) as e:
        for d in split_batches(stream, batches):
            engine_ingest(e, d, hashed=hashed)
        touched = [s for s in range(n_slots[3]) if w.touched(3, s)]
        if check_state:
            for s in touched:
                _set_state_equal(e, w, s)
        f = e.flush()
    assert f.set_slot.tolist() == touched
    exp = np.array([w.set_estimate(s) for s in touched], np.uint64)
    bad = np.nonzero(f.set_estimate != exp)[0]
    assert len(bad) == 0, [(touched[i], int(f.set_estimate[i]), int(exp[i])) for i in bad[:10]]
    return f


def test_set_random_members_parity():
    d = V.synth(seed=31, n_keys=500, zipf_s=1.1, mix=(0, 0, 0, 1), n_samples=200_000, member_universe=5_000_000)
    f = _set_parity(d, d["n_slots"])
    assert (f.set_sparse == 0).any() and (f.set_sparse == 1).any()  # both representations exercised


def test_set_random_members_parity_multi_batch():
    d = V.synth(seed=32, n_keys=200, zipf_s=1.2, mix=(0, 0, 0, 1), n_samples=120_000, member_universe=50_000)
    _set_parity(d, d["n_slots"], batches=5)


@pytest.mark.parametrize("batches", [1, 3])
def test_set_grouped_merges_and_dense_crossing(batches):
    """mergeSparse grouped over up to six triggers (ingest_set.hip, kSetGroup; hyperloglog.go:
    186-267): a key that stays sparse through many triggers, keys whose group's union passes m
    (its triggers scanned again one merge each, toNormal at the reference's record), a key whose
    list of 1-byte deltas leaves no room for a group, and repeated members across triggers."""
    rng = np.random.default_rng(61)
    parts = []
    # key 0: codes two apart (idx << 1, encodeHash with the top 25 bits = idx): 1-byte deltas, so
    # the list passes 13568 codes while sparse, then toNormal near 16384
    idx = rng.permutation(np.arange(1, 20001, dtype=np.uint64))
    parts.append((0, (idx << np.uint64(39)) | np.uint64(1 << 30)))
    parts.append((1, rng.integers(0, 2**63, 12000, dtype=np.uint64)))  # dense within the batch
    parts.append((2, rng.integers(0, 2**63, 3000, dtype=np.uint64)))   # sparse, ~18 triggers
    rep = rng.integers(0, 2**63, 2000, dtype=np.uint64)
    parts.append((3, rng.permutation(np.concatenate([rep, rep, rep]))))  # codes repeat across tmpSets
    slots = np.concatenate([np.full(len(h), k, np.uint32) for k, h in parts])
    hashes = np.concatenate([h for _, h in parts])
    order = rng.permutation(len(slots))  # keys interleaved; each key's own order is its arrival order
    d = {"c_slot": np.zeros(0, np.uint32), "c_val": np.zeros(0), "c_rate": np.zeros(0, np.float32),
         "g_slot": np.zeros(0, np.uint32), "g_val": np.zeros(0),
         "h_slot": np.zeros(0, np.uint32), "h_val": np.zeros(0), "h_rate": np.zeros(0, np.float32),
         "s_slot": slots[order], "s_hash": hashes[order]}
    w = run_oracle(d, (0, 0, 0, 4), hashed=True)
    assert not w.set_sketch(0).sparse and not w.set_sketch(1).sparse and w.set_sketch(2).sparse
    _set_parity(d, (1, 1, 1, 4), batches=batches, hashed=True)


def test_set_dense_rebase_epochs():
    """One key receives enough distinct hashes to fill all 16384 registers, then keeps going,
    so rebases (b > 0) happen mid-stream (hyperloglog.go:168-183, registers.go:55-123)."""
    rng = np.random.default_rng(41)
    n = 400_000
    hashes = rng.integers(0, 2**63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    slots = np.zeros(n, np.uint32)
    slots[::97] = 1  # a second, smaller key
    d = {"c_slot": np.zeros(0, np.uint32), "c_val": np.zeros(0), "c_rate": np.zeros(0, np.float32),
         "g_slot": np.zeros(0, np.uint32), "g_val": np.zeros(0),
         "h_slot": np.zeros(0, np.uint32), "h_val": np.zeros(0), "h_rate": np.zeros(0, np.float32),
         "s_slot": slots, "s_hash": hashes}
    w = run_oracle(d, (0, 0, 0, 2), hashed=True)
    assert w.set_sketch(0).b > 0  # the case is meaningful
    _set_parity(d, (1, 1, 1, 2), batches=3, hashed=True)


def test_set_crafted_rebase_cascade():
    """Hashes that fill every register with rho=2..3 quickly, then large-rho candidates and
    rho=1 inserts once b >= 2 (the wrapped uint8(r-b) candidates)."""
    rng = np.random.default_rng(42)
    idx = np.arange(16384, dtype=np.uint64)
    fill = (idx << np.uint64(50)) | (np.uint64(1) << np.uint64(48))     # rho = 2 for every register
    fill3 = (idx << np.uint64(50)) | (np.uint64(1) << np.uint64(47))    # rho = 3
    big = (rng.integers(0, 16384, 50, dtype=np.uint64) << np.uint64(50)) | np.uint64(1)  # rho = 50
    ones = (rng.integers(0, 16384, 3000, dtype=np.uint64) << np.uint64(50)) | (np.uint64(1) << np.uint64(49))
    rnd = rng.integers(0, 2**63, 60000, dtype=np.uint64)
    hashes = np.concatenate([fill, big[:10], fill3, big[10:30], ones, big[30:], rnd])
    hashes = np.concatenate([hashes, rng.permutation(hashes)])
    d = {"c_slot": np.zeros(0, np.uint32), "c_val": np.zeros(0), "c_rate": np.zeros(0, np.float32),
         "g_slot": np.zeros(0, np.uint32), "g_val": np.zeros(0),
         "h_slot": np.zeros(0, np.uint32), "h_val": np.zeros(0), "h_rate": np.zeros(0, np.float32),
         "s_slot": np.zeros(len(hashes), np.uint32), "s_hash": hashes}
    w = run_oracle(d, (0, 0, 0, 1), hashed=True)
    assert w.set_sketch(0).b >= 2
    _set_parity(d, (1, 1, 1, 1), batches=4, hashed=True)


# ------------------------------------------------------------------ mixed stream (C3 shape, small)
def test_mixed_stream_end_to_end():
    d = V.synth(seed=51, n_keys=3000, zipf_s=1.0, n_samples=300_000, member_universe=2_000_000)
    n_slots = d["n_slots"]
    w = run_oracle(d, n_slots)
    with make_engine(n_slots, max_records=1 << 19) as e:
        for b in split_batches(d, 3):
            engine_ingest(e, b)
        f = e.flush()
    assert f.samples_processed == 300_000
    exp_c = {s: w.counter_value(s) for s in range(n_slots[0]) if w.touched(0, s)}
    assert dict(zip(f.counter_slot.tolist(), f.counter_value.tolist())) == exp_c
    exp_g = {s: w.gauge_value(s) for s in range(n_slots[1]) if w.touched(1, s)}
    assert dict(zip(f.gauge_slot.tolist(), f.gauge_value.tolist())) == exp_g
    exp_s = {s: w.set_estimate(s) for s in range(n_slots[3]) if w.touched(3, s)}
    assert dict(zip(f.set_slot.tolist(), f.set_estimate.tolist())) == exp_s
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    assert rank_errors(d, f.histo_slot, f.histo_quantiles, oq).max() <= 1e-3


def test_flush_resets_window():  # worker.go:276-284: a new window starts empty
    with make_engine((2, 2, 2, 2)) as e:
        e.ingest(counters=([0], [1.0], [1.0]), histos=([1], [3.0], [1.0]),
                 set_hashes=(np.array([0], np.uint32), np.array([123456789], np.uint64)))
        f1 = e.flush()
        assert len(f1.counter_slot) == 1 and len(f1.histo_slot) == 1 and len(f1.set_slot) == 1
        f2 = e.flush()
        assert len(f2.counter_slot) == len(f2.histo_slot) == len(f2.set_slot) == len(f2.gauge_slot) == 0
        e.ingest(counters=([0], [2.0], [1.0]), histos=([1], [7.0], [1.0]))
        f3 = e.flush()
        assert f3.counter_value.tolist() == [2]
        assert f3.histo_stats[0][1] == 7.0 and f3.histo_quantiles[0][0] == 7.0


def test_invalid_inputs_fail_loudly():  # merging_digest.go:98-100 panics; parser rejects rates
    with make_engine((2, 2, 2, 2)) as e:
        with pytest.raises(V.EngineError):
            e.ingest(histos=([0], [float("nan")], [1.0]))
        with pytest.raises(V.EngineError):
            e.ingest(histos=([0], [1.0], [0.0]))
        with pytest.raises(V.EngineError):
            e.ingest(counters=([5], [1.0], [1.0]))  # slot out of range


def test_histo_quantile_cdf_queries():  # merging_digest.go:247-313 (Quantile, CDF mid-window)
    d = V.synth(seed=25, n_keys=60, zipf_s=1.0, mix=(0, 0, 1, 0), n_samples=40_000)
    w = run_oracle(d, d["n_slots"])
    rng = np.random.default_rng(3)
    with make_engine(d["n_slots"]) as e:
        engine_ingest(e, d)
        slots = np.array([s for s in range(d["n_slots"][2]) if w.touched(2, s)], np.uint32)
        xs = np.exp(rng.normal(3.9, 1.2, len(slots)))
        qs = rng.random(len(slots))
        got_c = e.cdf(slots, xs)
        got_q = e.quantile(slots, qs)
        with pytest.raises(V.EngineError):
            e.quantile(slots[:1], [1.5])  # Quantile panics outside [0, 1] (284-286)
        f = e.flush()  # the queries merged pending temps: flush quantiles are unchanged by them
    exp_c = np.array([w.histo_cdf(int(s), float(x)) for s, x in zip(slots, xs)])
    exp_q = np.array([w.histo_quantile(int(s), float(q)) for s, q in zip(slots, qs)])
    np.testing.assert_array_equal(got_c, exp_c)
    np.testing.assert_array_equal(got_q, exp_q)
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_quantiles, oq)


@FAST_ONLY
@pytest.mark.parametrize("batches", [5, 10])
def test_histo_keys_cross_threshold_across_batches(batches):
    """every key (~48k samples) passes the exact threshold in a later batch than its first (the
    import run's pattern): weights, min/max exact; the warm keys' rank error stays within the
    bound the single-batch scheme shows for keys just past the threshold"""
    d = V.synth(seed=25, n_keys=100, zipf_s=0.0, mix=(0, 0, 1, 0), n_samples=4_800_000)
    _histo_parity(d, d["n_slots"], batches=batches, max_rank=3e-3, exact_threshold=32768)


def test_histo_exact_replay_long_keys_multi_batch():
    """four-wave replays (a key's batch share of 65536 .. 524287 samples) continuing from pending
    temps, batch after batch: bit-identical quantiles"""
    d = V.synth(seed=26, n_keys=8, zipf_s=0.0, mix=(0, 0, 1, 0), n_samples=3_200_000)
    _histo_parity(d, d["n_slots"], batches=4, max_rank=0.0)


@FAST_ONLY
def test_histo_warm_keys_only_single_batch():
    """every key warm (E < n <= 4E) and none hot: the replay of E samples then the warm rounds,
    with no hot-prefix stream in the batch"""
    d = V.synth(seed=27, n_keys=16, zipf_s=0.0, mix=(0, 0, 1, 0), n_samples=1_280_000)
    _histo_parity(d, d["n_slots"], batches=1, max_rank=3e-3, exact_threshold=32768)


@FAST_ONLY
def test_histo_warm_imports_single_batch():
    """the same shape as imported centroids (Histo.Combine of many hosts' digests in one run)"""
    rng = np.random.default_rng(28)
    nk, hosts = 16, 800
    w = oracle.Worker(1, 1, nk, 1)
    with make_engine((1, 1, nk, 1), max_records=1 << 24, exact_threshold=32768) as e:
        for h in range(hosts):
            pay = []
            for k in range(nk):
                t = oracle.MergingDigest(100.0)
                n = int(rng.integers(50, 150))
                t.add_many(np.exp(rng.normal(3.9, 1.0, n)), np.where(rng.random(n) < 0.1, 2.0, 1.0))
                pay.append(t.gob_encode())
            e.import_histos(np.arange(nk, dtype=np.uint32), pay)
            for k in range(nk):
                assert w.import_histo(k, pay[k]) == 0
        f = e.flush()
    ost = np.array([w.histo_stats(k) for k in range(nk)])
    np.testing.assert_array_equal(f.histo_stats[:, [5, 6, 7]], ost[:, [5, 6, 7]])


def test_histo_duplicate_values_past_threshold():
    """integer-valued timers (every value repeated thousands of times) on warm and hot keys:
    the batch merge's centroid means stay ordered, so no element is lost (weights, min/max
    exact) and the rank error holds"""
    rng = np.random.default_rng(29)
    sizes = [60_000, 90_000, 300_000, 5_000]
    slot = np.concatenate([np.full(n, k, np.uint32) for k, n in enumerate(sizes)])
    rng.shuffle(slot)
    val = np.maximum(1.0, np.round(np.exp(rng.normal(3.0, 0.8, len(slot)))))
    rate = np.where(rng.random(len(slot)) < 0.1, np.float32(0.5), np.float32(1.0)).astype(np.float32)
    d = {"c_slot": np.zeros(0, np.uint32), "c_val": np.zeros(0), "c_rate": np.zeros(0, np.float32),
         "g_slot": np.zeros(0, np.uint32), "g_val": np.zeros(0), "h_slot": slot, "h_val": val, "h_rate": rate,
         "s_slot": np.zeros(0, np.uint32), "s_off": np.zeros(1, np.uint32), "s_bytes": np.zeros(0, np.uint8)}
    if V._abi.FAST_MODE:  # (the opt-in fast mode, a variant build)
        _histo_parity(d, (1, 1, len(sizes), 1), batches=3, max_rank=3e-3, exact_threshold=32768)
    _histo_parity(d, (1, 1, len(sizes), 1), batches=3, max_rank=0.0)  # the default: every merge replayed


@FAST_ONLY
def test_histo_hot_key_near_tie_values():
    """a hot key whose values share their top 40 ordered bits by the thousand (1000 + U(0, 1e-4):
    runs far longer than k_fix_ties sorts in place, not in full-value order) -- the tie check
    sets the device flag and the full-width re-sort of the remainder runs; rank error holds
    although every quantile sits inside a 1e-4 wide cluster"""
    rng = np.random.default_rng(31)
    sizes = [300_000, 50_000]
    slot = np.concatenate([np.full(n, k, np.uint32) for k, n in enumerate(sizes)])
    rng.shuffle(slot)
    val = np.where(slot == 0, 1000.0 + rng.random(len(slot)) * 1e-4, rng.lognormal(2.0, 1.0, len(slot)))
    rate = np.ones(len(slot), np.float32)
    d = {"c_slot": np.zeros(0, np.uint32), "c_val": np.zeros(0), "c_rate": np.zeros(0, np.float32),
         "g_slot": np.zeros(0, np.uint32), "g_val": np.zeros(0), "h_slot": slot, "h_val": val, "h_rate": rate,
         "s_slot": np.zeros(0, np.uint32), "s_off": np.zeros(1, np.uint32), "s_bytes": np.zeros(0, np.uint8)}
    _histo_parity(d, (1, 1, len(sizes), 1), batches=2, exact_threshold=20000)


def _c4_hot_stream(seed, sizes, rates=(1.0, 0.5, 0.1), noise_keys=200, noise=40_000):
    """histo keys with the window sizes of C4's hottest timers (slots 16 / 33 / 68 / 119 / 255
    hold 979k / 469k / 224k / 145k / 63k samples at N = 1), lognormal values, mixed sample rates,
    interleaved with a tail of small keys"""
    rng = np.random.default_rng(seed)
    slot = np.concatenate([np.full(n, k, np.uint32) for k, n in enumerate(sizes)] +
                          [rng.integers(len(sizes), len(sizes) + noise_keys, noise).astype(np.uint32)])
    rng.shuffle(slot)
    val = rng.lognormal(np.log(50.0), 1.0, len(slot))
    rate = np.asarray(rates, np.float32)[rng.choice(len(rates), len(slot), p=(0.9, 0.05, 0.05)[:len(rates)])]
    return {"c_slot": np.zeros(0, np.uint32), "c_val": np.zeros(0), "c_rate": np.zeros(0, np.float32),
            "g_slot": np.zeros(0, np.uint32), "g_val": np.zeros(0), "h_slot": slot, "h_val": val, "h_rate": rate,
            "s_slot": np.zeros(0, np.uint32), "s_off": np.zeros(1, np.uint32), "s_bytes": np.zeros(0, np.uint8)}


def test_histo_c4_hot_key_sizes_exact():
    """one 400k-sample lognormal key and keys of 250k / 145k / 63k / 40k
    samples (the C4 slots whose quantiles the geometric merge took past 1e-3), sample rates 1 /
    0.5 / 0.1, in two batches: the default mode replays every merge -- the four-wave long replay
    (replay_key_fast) for these keys -- so every quantile is the reference's, bit for bit"""
    sizes = [400_000, 250_000, 145_000, 63_000, 40_000]
    d = _c4_hot_stream(61, sizes)
    errs = _histo_parity(d, (1, 1, len(sizes) + 200, 1), batches=2, max_rank=0.0)
    assert errs.shape[0] >= len(sizes)


@FAST_ONLY
def test_histo_c4_hot_key_sizes_fast_mode_bound():
    """the same keys through the opt-in fast mode (geometric pieces past 32768 samples): within
    the 1e-3 bound only by luck of the order, so this checks the looser 3e-3 it documents"""
    sizes = [400_000, 250_000, 145_000, 63_000, 40_000]
    d = _c4_hot_stream(61, sizes)
    _histo_parity(d, (1, 1, len(sizes) + 200, 1), batches=2, max_rank=3e-3, exact_threshold=32768)
