"""Pins the CPU oracle to every known-answer vector the reference's own tests hold
for the sketch path.  CPU only.

Each test names the reference test it restates.
"""
import base64
import json
import os
import struct

import numpy as np
import pytest

import oracle
from oracle import MergingDigest, Sketch, decode_hash, encode_hash

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def nop_sketch(p):
    """NewTestSketch (hyperloglog_test.go:602-606): hash = nopHash, so Insert(toByte(v)) == insert_hash(v)."""
    return Sketch(p)


# ---------------------------------------------------------------- go-metro
def test_metro64_kat():  # vendor/github.com/dgryski/go-metro/metro_test.go:9-27
    key63 = b"012345678901234567890123456789012345678901234567890123456789012"
    want0 = struct.unpack("<Q", bytes([0x6B, 0x75, 0x3D, 0xAE, 0x06, 0x70, 0x4B, 0xAD]))[0]
    want1 = struct.unpack("<Q", bytes([0x3B, 0x0D, 0x48, 0x1C, 0xF4, 0xB9, 0xB8, 0xDF]))[0]
    assert oracle.metro64(key63, 0) == want0
    assert oracle.metro64(key63, 1) == want1


def test_clz():  # go-bits clz_amd64.s: BSR based, Clz(0) == 64
    assert oracle.lib.or_clz64(0) == 64
    assert oracle.lib.or_clz64(1) == 63
    assert oracle.lib.or_clz64(1 << 63) == 0


# ---------------------------------------------------------------- routing digest
def test_fnv_worker_routing_kat():  # http_test.go:23-32
    idx = [oracle.metric_digest(n, t) % 96 for n, t in
           (("foo", "histogram"), ("bar", "set"), ("baz", "counter"), ("qux", "gauge"))]
    assert idx == [0x4F, 0x3A, 0x2, 0x3C]


def test_fnv_parse_digest_matches_import_hash():  # http_test.go:43-57 ("foo:1|h|#bar")
    # ParseMetric writes name, "histogram", joined sorted tags; newSortableJSONMetrics writes
    # Name, Type, JoinedTags: identical bytes, identical digest.
    assert oracle.metric_digest("foo", "histogram", "bar") == oracle.fnv1a32(b"foo", b"histogram", b"bar")


# ---------------------------------------------------------------- HLL (nopHash KATs)
def test_hll_add_nosparse():  # hyperloglog_test.go:69-109
    sk = nop_sketch(16)
    sk.to_normal()
    sk.insert_hash(0x00010FFFFFFFFFFF)
    assert sk.reg_get(1) == 5
    sk.insert_hash(0x0002FFFFFFFFFFFF)
    assert sk.reg_get(2) == 1
    sk.insert_hash(0x0003000000000000)
    assert sk.reg_get(3) == 15
    sk.insert_hash(0x0003000000000001)
    assert sk.reg_get(3) == 15
    sk.insert_hash(0xFF03700000000000)
    assert sk.reg_get(0xFF03) == 2
    sk.insert_hash(0xFF03080000000000)
    assert sk.reg_get(0xFF03) == 5


def test_hll_precision_nosparse():  # hyperloglog_test.go:111-132
    sk = nop_sketch(4)
    sk.to_normal()
    sk.insert_hash(0x1FFFFFFFFFFFFFFF)
    assert sk.reg_get(1) == 1
    sk.insert_hash(0xFFFFFFFFFFFFFFFF)
    assert sk.reg_get(0xF) == 1
    sk.insert_hash(0x00FFFFFFFFFFFFFF)
    assert sk.reg_get(0) == 5


def test_hll_to_normal():  # hyperloglog_test.go:134-173
    sk = nop_sketch(16)
    sk.insert_hash(0x00010FFFFFFFFFFF)
    sk.to_normal()
    assert sk.estimate() == 1
    assert not sk.sparse
    sk = nop_sketch(16)
    for v in (0x00010FFFFFFFFFFF, 0x0002FFFFFFFFFFFF, 0x0003000000000000, 0x0003000000000001,
              0xFF03700000000000, 0xFF03080000000000):
        sk.insert_hash(v)
    sk.merge_sparse()
    sk.to_normal()
    assert sk.reg_get(1) == 5
    assert sk.reg_get(2) == 1
    assert sk.reg_get(3) == 15
    assert sk.reg_get(0xFF03) == 5


def test_hll_cardinality():  # hyperloglog_test.go:175-208
    sk = nop_sketch(16)
    assert sk.estimate() == 0
    for v in (0x00010FFFFFFFFFFF, 0x00020FFFFFFFFFFF, 0x00030FFFFFFFFFFF, 0x00040FFFFFFFFFFF,
              0x00050FFFFFFFFFFF, 0x00050FFFFFFFFFFF):
        sk.insert_hash(v)
    assert sk.estimate() == 5
    assert sk.estimate() == 5
    sk.insert_hash(0x00060FFFFFFFFFFF)
    assert sk.estimate() == 6


def test_hll_merge_error():  # hyperloglog_test.go:210-218
    with pytest.raises(ValueError):
        nop_sketch(16).merge(nop_sketch(10))


def test_hll_merge_sparse():  # hyperloglog_test.go:220-272
    sk = nop_sketch(16)
    for v in (0x00010FFFFFFFFFFF, 0x00020FFFFFFFFFFF, 0x00030FFFFFFFFFFF, 0x00040FFFFFFFFFFF,
              0x00050FFFFFFFFFFF, 0x00050FFFFFFFFFFF):
        sk.insert_hash(v)
    sk2 = nop_sketch(16)
    sk2.merge(sk)
    assert sk2.estimate() == 5
    assert sk2.sparse and sk.sparse
    sk2.merge(sk)
    assert sk2.estimate() == 5
    for v in (0x00060FFFFFFFFFFF, 0x00070FFFFFFFFFFF, 0x00080FFFFFFFFFFF, 0x00090FFFFFFFFFFF,
              0x000A0FFFFFFFFFFF, 0x000A0FFFFFFFFFFF):
        sk.insert_hash(v)
    assert sk.estimate() == 10
    sk2.merge(sk)
    assert sk2.estimate() == 10


def test_hll_merge_rebase():  # hyperloglog_test.go:274-319
    sk1, sk2 = nop_sketch(16), nop_sketch(16)
    sk1.sparse = False
    sk2.sparse = False
    sk1.to_normal()
    sk2.to_normal()
    sk1.reg_set(13, 7)
    sk2.reg_set(13, 1)
    sk1.merge(sk2)
    assert sk1.reg_get(13) == 7
    sk2.reg_set(13, 8)
    sk1.merge(sk2)
    assert sk2.reg_get(13) == 8
    assert sk1.reg_get(13) == 8
    sk1.b = 12
    sk2.reg_set(13, 12)
    sk1.merge(sk2)
    assert sk1.reg_get(13) == 8
    sk2.b = 13
    sk2.reg_set(13, 12)
    sk1.merge(sk2)
    assert sk1.reg_get(13) == 12


def test_hll_encode_decode():  # hyperloglog_test.go:388-429
    p = 8
    assert decode_hash(encode_hash(0xFFFFFF8000000000, p), p) == (0xFF, 1)
    assert decode_hash(encode_hash(0xFF00000000000000, p), p) == (0xFF, 57)
    assert decode_hash(encode_hash(0xFF30000000000000, p), p) == (0xFF, 3)
    assert decode_hash(encode_hash(0xAA10000000000000, p), p) == (0xAA, 4)
    assert decode_hash(encode_hash(0xAA0F000000000000, p), p) == (0xAA, 5)


def test_hll_decode_encode_equals_getposval():
    """SURVEY H-4: decode(encode(x)) == getPosVal(x) at p=14, pp=25 (what the engine relies on)."""
    rng = np.random.default_rng(1)
    xs = list(rng.integers(0, 2**63, 4000, dtype=np.uint64) * 2 + rng.integers(0, 2, 4000, dtype=np.uint64))
    xs += [0, 1, (1 << 64) - 1, 1 << 39, (1 << 39) - 1, 0x0000008000000000, 0xFFFF800000000000]
    xs += [int(v) & ~((1 << 50) - 1) for v in xs[:500]]  # zero low bits -> exercise large rho
    xs += [int(v) & ~(0x7FF << 39) for v in xs[:500]]  # 11 bits after the index zero -> odd codes
    for x in xs:
        x = int(x)
        assert decode_hash(encode_hash(x, 14), 14) == oracle.get_pos_val(x, 14)


def test_hll_error():  # hyperloglog_test.go:431-446
    with pytest.raises(ValueError):
        Sketch(3)
    Sketch(18)
    with pytest.raises(ValueError):
        Sketch(19)


def test_hll_marshal_unmarshal_sparse():  # hyperloglog_test.go:448-478
    sk = Sketch(4)
    sk.tmp_add(26)
    sk.tmp_add(40)
    rng = np.random.default_rng(7)
    for v in rng.integers(0, 2**32, 10):
        sk.list_append(int(v))
    data = sk.marshal()
    assert data[0] == 1
    res = Sketch(14)
    res.unmarshal(data)
    assert res.sparse and res.p == 4 and res.b == 0
    assert list(res.tmp_codes()) == [26, 40]
    assert res.list_count() == sk.list_count() and res.list_bytes() == sk.list_bytes()
    assert res.marshal() == data


def test_hll_marshal_unmarshal_dense():  # hyperloglog_test.go:480-510
    sk = Sketch(4)
    sk.sparse = False
    sk.to_normal()
    rng = np.random.default_rng(3)
    for i in range(10):
        sk.reg_set(i, int(rng.integers(0, 256)))
    data = sk.marshal()
    assert data[0] == 1
    res = Sketch(14)
    res.unmarshal(data)
    assert not res.sparse
    assert res.marshal() == data
    assert np.array_equal(res.registers(), sk.registers())


def test_hll_clone():  # hyperloglog_test.go:561-584
    sk1 = nop_sketch(16)
    for v in (0x00010FFFFFFFFFFF, 0x0002FFFFFFFFFFFF, 0x0003000000000000, 0x0003000000000001, 0xFF03700000000000):
        sk1.insert_hash(v)
    assert sk1.estimate() == 5
    sk2 = sk1.clone()
    assert sk1.estimate() == sk2.estimate()
    assert sk1.marshal() == sk2.marshal()
    sk1.to_normal()
    sk2 = sk1.clone()
    assert sk1.estimate() == sk2.estimate()
    assert sk1.marshal() == sk2.marshal()


def test_registers_zeros():  # registers_test.go:27-54
    sk = Sketch(4)  # only the register file is exercised; m = 8 registers via p=... use rebase on p=4
    sk.sparse = False
    sk.to_normal()
    # registers_test uses newRegisters(8); the first 8 registers of a p=4 sketch behave identically
    # except for nz, which counts all 16.  Fill every register so nz reflects only the first 8 rule.
    for i in range(16):
        sk.reg_set(i, (i % 15) + 1)
    for i in range(16):
        sk.reg_set(i, (i % 15) + 1)
    for i in range(16):
        assert sk.reg_get(i) == (i % 15) + 1
    sk.reg_rebase(1)
    for i in range(16):
        assert sk.reg_get(i) == i % 15
    # registers 0 and 15 become zero: nz counts them (registers_test: m=8 -> only register 0 -> 1)
    assert sk.nz == 2


def test_hll_cardinality_hashed():  # hyperloglog_test.go:31-61 (1e6 here; the reference runs 1e7)
    sk = Sketch(14)
    unique = 0
    step = 10
    for i in range(1, 1_000_001):
        sk.insert(b"flow-%d" % i)
        unique += 1
        if unique % step == 0:
            step *= 5
            est = sk.estimate()
            assert abs(est - unique) / unique <= 0.02, (unique, est)
    est = sk.estimate()
    assert abs(est - unique) / unique <= 0.02


# ---------------------------------------------------------------- samplers KATs
def test_set_kat():  # samplers_test.go:144-168
    w = oracle.Worker(1, 1, 1, 1)
    members = [b"5", b"5", b"123", b"2147483647", b"-2147483648"]
    off = np.cumsum([0] + [len(m) for m in members]).astype(np.uint32)
    w.set(np.zeros(len(members), np.uint32), off, np.frombuffer(b"".join(members), np.uint8))
    assert w.set_estimate(0) == 4


def test_counter_kats():  # samplers_test.go:46-106
    w = oracle.Worker(4, 0, 0, 0)
    w.counter([0], [1.0], [1.0])
    w.counter([1], [5.0], [1.0])
    w.counter([2], [5.0], [0.5])
    assert [w.counter_value(s) for s in range(3)] == [1, 5, 10]
    # CounterMerge: export 5@0.5 (=10) and 14@0.5 (=28) into a global counter
    w.import_counter(3, 10)
    assert w.counter_value(3) == 10
    w.import_counter(3, 28)
    assert w.counter_value(3) == 38


def test_counter_float32_truncation():  # samplers.go:133 (float32 1/rate, then int64)
    w = oracle.Worker(3, 0, 0, 0)
    w.counter([0], [3.7], [np.float32(0.3)])   # int64(3.7)=3, float32(1/0.3)=3.3333333 -> 3
    w.counter([1], [-2.9], [np.float32(0.1)])  # -2 * 10
    w.counter([2], [1e300], [1.0])              # out of int64 range -> amd64 integer indefinite
    assert w.counter_value(0) == 9
    assert w.counter_value(1) == -20
    assert w.counter_value(2) == -(1 << 63)


def test_gauge_kat():  # samplers_test.go:108-142
    w = oracle.Worker(0, 2, 0, 0)
    w.gauge([0], [5.0])
    assert w.gauge_value(0) == 5.0
    w.import_gauge(1, 1.0)
    w.import_gauge(1, 5.0)
    assert w.gauge_value(1) == 5.0


def test_histo_kat():  # samplers_test.go:192-283
    w = oracle.Worker(0, 0, 1, 0)
    w.histo([0] * 5, [5, 10, 15, 20, 25], [1.0] * 5)
    st = w.histo_stats(0)
    assert st[2] == 25 and st[1] == 5 and st[3] == 75
    assert st[3] / st[0] == 15 and st[0] == 5
    assert w.histo_quantile(0, 0.5) == 15
    assert st[0] / st[4] == 5.0 / ((1.0 / 5) + (1.0 / 10) + (1.0 / 15) + (1.0 / 20) + (1.0 / 25))
    assert w.histo_quantile(0, 0.90) == 23.75


def test_histo_sample_rate():  # samplers_test.go:354-382
    w = oracle.Worker(0, 0, 1, 0)
    w.histo([0] * 5, [5, 10, 15, 20, 25], [0.5] * 5)
    st = w.histo_stats(0)
    assert st[2] == 25 and st[0] == 10


# ---------------------------------------------------------------- t-digest
def test_tdigest_fixture_decode_and_quantiles():
    """fixtures/import.uncompressed == server_test.go:308 ExpectedGobStream: centroids {1,2,7,8,100},
    delta=100, min 1, max 100.  Quantiles (server_test.go:121-138 lists 6/42/98 as approximations)."""
    items = json.load(open(os.path.join(GOLD, "import.uncompressed")))
    gob = base64.b64decode(items[0]["value"])
    assert gob == open(os.path.join(GOLD, "tdigest_1_2_7_8_100.gob"), "rb").read()
    td = MergingDigest(100)
    td.gob_decode(gob)
    m, w = td.centroids()
    assert list(m) == [1, 2, 7, 8, 100] and list(w) == [1] * 5
    assert td.min() == 1 and td.max() == 100 and td.count() == 5
    assert td.quantile(0.5) == 6
    assert td.quantile(0.75) == 42.375
    assert td.quantile(0.99) == pytest.approx(97.7, rel=1e-15)


def test_tdigest_gob_encode_reproduces_fixture():  # TestLocalServerMixedMetrics (server_test.go:303-416)
    td = MergingDigest(100)
    for v in (1.0, 2.0, 7.0, 8.0, 100.0):
        td.add(v, 1.0)
    assert td.gob_encode() == open(os.path.join(GOLD, "tdigest_1_2_7_8_100.gob"), "rb").read()


def _validate(td, compression):  # histo_test.go:46-66 (validateMergingDigest)
    m, w = td.centroids()
    total = w.sum()
    k = lambda q: compression * (np.arcsin(2 * q - 1) / np.pi + 0.5)
    index, q = 0.0, 0.0
    for i in range(len(m)):
        nxt = k(min(1.0, q + w[i] / total))
        if 0 < i < len(m) - 1:
            assert nxt - index <= 1 + 1e-9 or w[i] == 1, "centroid is oversized"
        q += w[i] / total
        index = nxt
    assert total == td.count()


def test_tdigest_accuracy():  # histo_test.go:11-25
    rng = np.random.default_rng(11)
    td = MergingDigest(1000)
    for v in rng.random(200_000):
        td.add(float(v), 1.0)
    _validate(td, 1000)
    assert td.quantile(0.5) == pytest.approx(0.5, rel=0.02)
    assert td.min() >= 0 and td.max() < 1


def test_tdigest_merge_sparse():  # histo_test.go:27-41
    td = MergingDigest(1000)
    td.add(-200000, 1)
    other = MergingDigest(1000)
    other.add(200000, 1)
    td.merge(other)
    assert td.cdf(0) == pytest.approx(0.5, rel=0.02)
    assert abs(td.quantile(0.5)) <= 0.02
    assert td.quantile(0) == pytest.approx(td.min(), rel=0.02)
    assert td.quantile(1) == pytest.approx(td.max(), rel=0.02)


def test_tdigest_gob_roundtrip():  # histo_test.go:68-87
    rng = np.random.default_rng(5)
    td = MergingDigest(1000)
    for v in rng.random(1000):
        td.add(float(v), 1.0)
    td2 = MergingDigest(1000)
    td2.gob_decode(td.gob_encode())
    assert td2.count() == td.count() and td2.min() == td.min() and td2.max() == td.max()
    assert td2.quantile(0.5) == td.quantile(0.5)


def test_tdigest_invalid_add():  # merging_digest.go:98-100 (panic)
    td = MergingDigest(100)
    for v, w in ((float("nan"), 1), (float("inf"), 1), (1.0, 0.0), (1.0, -1)):
        with pytest.raises(ValueError):
            td.add(v, w)


def test_go_math_log_pow_known_values():
    # exactly representable results of the restated Go routines
    assert oracle.lib.or_go_log(1.0) == 0.0
    assert oracle.lib.or_go_pow(2.0, 10.0) == 1024.0
    assert oracle.lib.or_go_pow(0.0, 3.0) == 0.0
    assert oracle.lib.or_go_log(2.0) == pytest.approx(np.log(2.0), rel=1e-16, abs=0)
    xs = np.random.default_rng(0).random(1000) * 20
    for x in xs:
        assert oracle.lib.or_go_log(float(x)) == pytest.approx(np.log(x), rel=2e-16)
        assert oracle.lib.or_go_asin(float(x / 20)) == pytest.approx(np.arcsin(x / 20), rel=1e-15)


# ---------------------------------------------------------------- NaN sample rates
def _merge_all_temps_bounded(main, temps, main_weight, max_steps):
    """mergeAllTemps (merging_digest.go:121-205) restated loop for loop over (mean, weight) pairs,
    with a step bound: returns (new main, new main weight) or None when the loop has run
    max_steps iterations without ending.  indexEstimate's asin is math.asin (NaN in, NaN out)."""
    import math
    temps = sorted(temps, key=lambda c: c[0])
    total = main_weight + sum(w for _, w in temps)  # td.mainWeight + td.tempWeight
    k = lambda q: 100.0 * (math.asin(2 * q - 1) / math.pi + 0.5) if q == q and -1 <= 2 * q - 1 <= 1 else float("nan")
    out, merged_w, last_idx = [], 0.0, 0.0

    def merge_one(before, nxt, before_idx):  # mergeOne, merging_digest.go:210-236
        if (k((before + nxt[1]) / total) - before_idx > 1) or not out:
            out.append(list(nxt))
            return k(before / total)
        c = out[-1]
        c[1] += nxt[1]
        c[0] += (nxt[0] - c[0]) * nxt[1] / c[1]
        return before_idx

    actual, swapped, ti, steps = list(main), [], 0, 0
    while len(actual) + len(swapped) != 0 or ti < len(temps):
        steps += 1
        if steps > max_steps:
            return None
        nt = temps[ti] if ti < len(temps) else (float("inf"), 0.0)
        nm = swapped[0] if swapped else (actual[0] if actual else (float("inf"), 0.0))
        if nm[0] < nt[0]:
            if actual:
                if swapped:
                    swapped = swapped[1:] + [actual[0]]
                actual = actual[1:]
            else:
                swapped = swapped[1:]
            last_idx = merge_one(merged_w, nm, last_idx)
            merged_w += nm[1]
        else:
            if actual:
                swapped.append(actual[0])
                actual = actual[1:]
            ti += 1
            last_idx = merge_one(merged_w, nt, last_idx)
            merged_w += nt[1]
    return [tuple(c) for c in out], total


def test_nan_weight_merge_never_ends():
    """Why a histogram sample with a NaN rate is refused ("NaN sample rates").

    The parser lets @nan through (parser.go:262-272: both comparisons false); Histo.Sample's weight
    float64(1/NaN) is NaN and MergingDigest.Add accepts it (merging_digest.go:98 checks weight <= 0).
    The merge that takes it has totalWeight NaN, so mergeOne never starts a new centroid: every
    element joins the first, whose mean turns NaN.  At the next mergeAllTemps the main centroid's
    NaN mean loses every `nextMain.Mean < nextTemp.Mean` test -- also against the +Inf sentinel
    once the temps are used up -- so it is never consumed and the loop never ends: Go's worker
    spins holding its mutex.  No output exists to match; the engine refuses the record and the
    Worker drops it (counted).  The restated loop is checked on a normal digest first."""
    ok = _merge_all_temps_bounded([], [(float(v), 1.0) for v in range(42)], 0.0, 10_000)
    assert ok is not None and len(ok[0]) > 1 and ok[1] == 42.0
    # 41 samples at rate 1 and one at rate NaN: the first merge collapses them into one NaN centroid
    temps = [(float(v), 1.0) for v in range(41)] + [(17.5, float("nan"))]
    first = _merge_all_temps_bounded([], temps, 0.0, 10_000)
    assert first is not None and len(first[0]) == 1
    (mean, weight), = first[0]
    assert mean != mean and weight != weight and first[1] != first[1]
    # the next 42 samples' merge: bounded at 100k steps against the ~43 a merge needs
    assert _merge_all_temps_bounded(first[0], [(float(v), 1.0) for v in range(42)], first[1], 100_000) is None
    # a counter's NaN rate is defined: int64(float32(1/NaN)) = MinInt64 on amd64, times the
    # truncated sample, wrapping (samplers.go:133)
    w = oracle.Worker(3, 0, 0, 0)
    w.counter([0, 1, 2], [2.0, 3.0, 5.0], np.array([np.nan, np.nan, 0.0], np.float32))
    assert [w.counter_value(s) for s in range(3)] == [0, -(1 << 63), -(1 << 63)]
