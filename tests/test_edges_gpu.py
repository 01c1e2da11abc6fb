"""Edge cases of the engine's boundary and of the per-key state machines, against the oracle:
empty batches and windows, batches of exactly max_batch_records, slots at the capacity edge,
t-digest keys around the 42-entry temp buffer (estimateTempBuffer(100), merging_digest.go:87-93),
empty and long set members, a key touched only by imports."""
import numpy as np
import pytest

import oracle
import veneur_amd as V
from tests.util import PCT, run_oracle

pytestmark = pytest.mark.gpu

Z32, ZF, ZF32 = np.zeros(0, np.uint32), np.zeros(0), np.zeros(0, np.float32)


def make_engine(n_slots, max_records=1 << 14):
    return V.Engine(tuple(n_slots), percentiles=PCT, max_batch_records=max_records,
                    max_batch_member_bytes=max_records * 64)


def stream(**kw):
    d = {"c_slot": Z32, "c_val": ZF, "c_rate": ZF32, "g_slot": Z32, "g_val": ZF, "h_slot": Z32, "h_val": ZF,
         "h_rate": ZF32, "s_slot": Z32, "s_off": np.zeros(1, np.uint32), "s_bytes": np.zeros(0, np.uint8)}
    d.update(kw)
    return d


def test_empty_batches_and_empty_window():
    with make_engine((4, 4, 4, 4)) as e:
        e.ingest()
        e.ingest(counters=(Z32, ZF, ZF32), gauges=(Z32, ZF), histos=(Z32, ZF, ZF32), set_hashes=(Z32, Z32.astype(np.uint64)))
        f = e.flush()
        assert (len(f.counter_slot), len(f.gauge_slot), len(f.histo_slot), len(f.set_slot)) == (0, 0, 0, 0)
        assert f.samples_processed == 0 and f.samples_imported == 0
        f = e.flush()  # a second empty window
        assert len(f.histo_slot) == 0


def test_batch_of_exactly_max_records_and_capacity_edges():
    n, cap = 1 << 14, 1000
    rng = np.random.default_rng(5)
    slots = rng.integers(0, cap, n).astype(np.uint32)
    slots[:4] = cap - 1  # the last slot of every class
    vals = np.round(rng.lognormal(3, 1, n), 3)
    rates = np.where(rng.random(n) < 0.2, np.float32(0.1), np.float32(1.0)).astype(np.float32)
    members = [("m%d" % i).encode() for i in rng.integers(0, 5000, n)]
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum([len(m) for m in members])
    mb = np.frombuffer(b"".join(members), np.uint8)
    d = stream(c_slot=slots, c_val=vals, c_rate=rates, g_slot=slots, g_val=vals, h_slot=slots, h_val=vals,
               h_rate=rates, s_slot=slots, s_off=off, s_bytes=mb)
    w = run_oracle(d, (cap,) * 4)
    with make_engine((cap,) * 4, max_records=n) as e:
        e.ingest(counters=(slots, vals, rates), gauges=(slots, vals), histos=(slots, vals, rates), sets=(slots, off, mb))
        with pytest.raises(V.EngineError):  # one record over max_batch_records fails loudly
            e.ingest(counters=(np.zeros(n + 1, np.uint32), np.ones(n + 1), np.ones(n + 1, np.float32)))
        with pytest.raises(V.EngineError):  # slot == capacity
            e.ingest(gauges=(np.array([cap], np.uint32), np.ones(1)))
        f = e.flush()
    assert f.samples_processed == 4 * n
    assert cap - 1 in f.counter_slot.tolist()
    assert dict(zip(f.counter_slot.tolist(), f.counter_value.tolist())) == \
        {s: w.counter_value(s) for s in range(cap) if w.touched(0, s)}
    assert dict(zip(f.gauge_slot.tolist(), f.gauge_value.tolist())) == \
        {s: w.gauge_value(s) for s in range(cap) if w.touched(1, s)}
    assert f.set_estimate.tolist() == [w.set_estimate(int(s)) for s in f.set_slot]
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_quantiles, oq)


@pytest.mark.parametrize("batches", [1, 3])
def test_digest_sizes_around_the_temp_buffer(batches):
    """Keys with 1, 41, 42, 43, 84, 85, 126, 127 and 1000 samples: every merge boundary of the
    42-entry temp buffer, within one batch and split across batches."""
    sizes = [1, 41, 42, 43, 84, 85, 126, 127, 1000]
    rng = np.random.default_rng(9)
    slots = np.concatenate([np.full(n, i, np.uint32) for i, n in enumerate(sizes)])
    perm = rng.permutation(len(slots))
    slots = slots[perm]
    vals = np.round(rng.lognormal(2, 1, len(slots)), 2)  # repeated values: ties in the temp sort
    rates = np.ones(len(slots), np.float32)
    w = oracle.Worker(1, 1, len(sizes), 1)
    w.histo(slots, vals, rates)
    with make_engine((1, 1, len(sizes), 1)) as e:
        for part in np.array_split(np.arange(len(slots)), batches):
            e.ingest(histos=(slots[part], vals[part], rates[part]))
        f = e.flush()
    assert f.histo_slot.tolist() == list(range(len(sizes)))
    ost = np.array([w.histo_stats(s) for s in range(len(sizes))])
    np.testing.assert_array_equal(f.histo_stats[:, [0, 1, 2, 5, 6, 7]], ost[:, [0, 1, 2, 5, 6, 7]])
    np.testing.assert_array_equal(f.histo_quantiles, [[w.histo_quantile(s, p) for p in PCT] for s in range(len(sizes))])


def test_set_members_empty_and_long():
    members = [b"", b"", b"x", b"a" * 4097, b"a" * 4097, bytes(range(256)) * 3, b"\x00"]
    slots = np.array([0, 0, 0, 0, 1, 1, 1], np.uint32)
    off = np.zeros(len(members) + 1, np.uint32)
    off[1:] = np.cumsum([len(m) for m in members])
    mb = np.frombuffer(b"".join(members), np.uint8)
    w = oracle.Worker(1, 1, 1, 2)
    w.set(slots, off, mb)
    with make_engine((1, 1, 1, 2)) as e:
        e.ingest(sets=(slots, off, mb))
        for s in (0, 1):
            assert np.array_equal(e.read_set(s)["tmp"], w.set_sketch(s).tmp_codes())
        f = e.flush()
    assert f.set_estimate.tolist() == [w.set_estimate(0), w.set_estimate(1)] == [3, 3]


def test_key_touched_only_by_imports():  # worker.go:237-242: imports Upsert the key too
    td = oracle.MergingDigest(100.0)
    td.add_many(np.arange(1.0, 50.0), np.ones(49))
    sk = oracle.Sketch()
    for h in range(1, 30):
        sk.insert_hash(h * 0x9E3779B97F4A7C15 % (1 << 64))
    hp, sp = td.gob_encode(), sk.marshal()
    w = oracle.Worker(2, 2, 2, 2)
    assert w.import_histo(1, hp) == 0
    w.import_set(1, sp)
    with make_engine((2, 2, 2, 2)) as e:
        e.import_counters(np.array([1], np.uint32), np.array([-7], np.int64))
        e.import_gauges(np.array([1], np.uint32), np.array([2.5]))
        e.import_histos(np.array([1], np.uint32), [hp])
        e.import_sets(np.array([1], np.uint32), [sp])
        f = e.flush()
    assert f.counter_slot.tolist() == [1] and f.counter_value.tolist() == [-7]
    assert f.gauge_value.tolist() == [2.5]
    assert f.histo_stats[0][0] == 0.0  # no local samples: LocalWeight stays 0 (samplers.go:519-526)
    assert f.histo_quantiles[0].tolist() == [w.histo_quantile(1, p) for p in PCT]
    assert f.set_estimate.tolist() == [w.set_estimate(1)]
    assert f.samples_imported == 4 and f.samples_processed == 0


def _device_batch(bufs, misalign=False, **cls):
    """An A.Batch whose arrays are copied to device memory (kept alive in bufs); misalign: every
    array starts one element past a 16-byte boundary (the validator's scalar path)."""
    import veneur_amd._abi as A

    def dev(a):
        if misalign:
            b = V.DeviceBuffer(np.concatenate([a[:1], a]))
            bufs.append(b)
            return b.ptr.value + a.itemsize
        b = V.DeviceBuffer(a)
        bufs.append(b)
        return b.ptr.value

    b = A.Batch()
    if "counters" in cls:
        s, v, r = cls["counters"]
        b.n_counter, b.counter_slot, b.counter_value, b.counter_rate = len(s), dev(s), dev(v), dev(r)
    if "gauges" in cls:
        s, v = cls["gauges"]
        b.n_gauge, b.gauge_slot, b.gauge_value = len(s), dev(s), dev(v)
    if "histos" in cls:
        s, v, r = cls["histos"]
        b.n_histo, b.histo_slot, b.histo_value, b.histo_rate = len(s), dev(s), dev(v), dev(r)
    if "sets" in cls:
        s, o, m = cls["sets"]
        b.n_set, b.set_slot, b.set_member_off, b.set_member_bytes = len(s), dev(s), dev(o), dev(m)
    return b


@pytest.mark.parametrize("where", ["mid", "quad_lane3", "tail", "misaligned"])
@pytest.mark.parametrize("fault", ["counter_slot", "gauge_slot", "histo_slot", "set_slot", "histo_nan",
                                   "histo_inf", "histo_rate_zero", "histo_rate_nan", "set_offsets"])
def test_device_batch_validation_rejects_and_leaves_state(fault, where):
    """vn_ingest validates a device-resident batch before applying anything (VN_EINVAL): a fault in
    a 16-byte quad (either lane), in the records past the last full quad, or in arrays that are not
    16-byte aligned (scalar checks)."""
    n, cap = 4099, 64
    rng = np.random.default_rng(3)
    slots = rng.integers(0, cap, n).astype(np.uint32)
    vals = np.round(rng.lognormal(3, 1, n), 3)
    rates = np.ones(n, np.float32)
    members = [("m%d" % i).encode() for i in rng.integers(0, 500, n)]
    off = np.zeros(n + 1, np.uint32)
    off[1:] = np.cumsum([len(m) for m in members])
    mb = np.frombuffer(b"".join(members), np.uint8).copy()
    good = dict(counters=(slots, vals, rates), gauges=(slots, vals), histos=(slots, vals, rates),
                sets=(slots, off, mb))
    bad = {k: tuple(a.copy() for a in v) for k, v in good.items()}
    i = {"mid": n // 2 - 1, "quad_lane3": n // 2 + 1, "tail": n - 2, "misaligned": n // 2}[where]
    if fault.endswith("_slot"):
        bad[{"counter": "counters", "gauge": "gauges", "histo": "histos", "set": "sets"}[fault[:-5]]][0][i] = cap
    elif fault == "histo_nan":
        bad["histos"][1][i] = np.nan
    elif fault == "histo_inf":
        bad["histos"][1][i] = -np.inf
    elif fault == "histo_rate_zero":
        bad["histos"][2][i] = 0.0
    elif fault == "histo_rate_nan":
        bad["histos"][2][i] = np.nan
    elif fault == "set_offsets":
        bad["sets"][1][i] = bad["sets"][1][i + 1] + 1
    bufs = []
    with make_engine((cap,) * 4) as e, make_engine((cap,) * 4) as ref:
        mis = where == "misaligned"
        e.ingest_device(_device_batch(bufs, misalign=mis, **good))
        with pytest.raises(V.EngineError, match="out of range|invalid value|sample rate|offsets"):
            e.ingest_device(_device_batch(bufs, misalign=mis, **bad))
        ref.ingest(**good)
        fe, fr = e.flush(), ref.flush()
    for b in bufs:
        b.free()
    assert fe.samples_processed == fr.samples_processed == 4 * n
    np.testing.assert_array_equal(fe.counter_value, fr.counter_value)
    np.testing.assert_array_equal(fe.gauge_value, fr.gauge_value)
    np.testing.assert_array_equal(fe.histo_quantiles, fr.histo_quantiles)
    np.testing.assert_array_equal(fe.histo_stats, fr.histo_stats)
    np.testing.assert_array_equal(fe.set_estimate, fr.set_estimate)


def test_submit_counter_only_batch_then_refill_stage():
    """vn_submit returns once the pinned stage has been copied: refilling it at once for the next
    batch (as the cgo binding in INTEGRATION.md does) cannot change what the first one ingested."""
    rng = np.random.default_rng(11)
    batches = [(rng.integers(0, 100, 50000).astype(np.uint32), rng.integers(1, 10, 50000).astype(np.float64))
               for _ in range(4)]
    with make_engine((100, 1, 1, 1), max_records=1 << 16) as e:
        st = e.stage()
        for s, v in batches:
            st["counter_slot"][:len(s)] = s
            st["counter_value"][:len(s)] = v
            st["counter_rate"][:len(s)] = 1.0
            e.submit(n_counter=len(s))
        f = e.flush()
    exp = np.zeros(100, np.int64)
    for s, v in batches:
        np.add.at(exp, s, v.astype(np.int64))
    assert f.counter_slot.tolist() == np.nonzero(exp)[0].tolist()
    np.testing.assert_array_equal(f.counter_value, exp[f.counter_slot])


def test_per_class_record_caps():
    """vn_config.max_batch_class_records: each class's batch is held to its own cap (its buffers
    are sized by it); a class cap above max_batch_records is refused at creation."""
    caps, cls = (64,) * 4, (300, 200, 500, 100)
    rng = np.random.default_rng(11)

    def recs(n):
        return rng.integers(0, 64, n).astype(np.uint32), np.round(rng.lognormal(2, 1, n), 3)

    cs, cv = recs(cls[0])
    gs, gv = recs(cls[1])
    hs, hv = recs(cls[2])
    ss, _ = recs(cls[3])
    members = [("u%d" % i).encode() for i in rng.integers(0, 1000, cls[3])]
    off = np.zeros(cls[3] + 1, np.uint32)
    off[1:] = np.cumsum([len(m) for m in members])
    mb = np.frombuffer(b"".join(members), np.uint8)
    one = lambda n: np.ones(n, np.float32)
    d = stream(c_slot=cs, c_val=cv, c_rate=one(len(cs)), g_slot=gs, g_val=gv, h_slot=hs, h_val=hv,
               h_rate=one(len(hs)), s_slot=ss, s_off=off, s_bytes=mb)
    w = run_oracle(d, caps)
    with V.Engine(caps, percentiles=PCT, max_batch_records=512, max_batch_member_bytes=1 << 16,
                  max_class_records=cls) as e:
        assert e.max_class_records == cls
        # every class at exactly its cap
        e.ingest(counters=(cs, cv, one(len(cs))), gauges=(gs, gv), histos=(hs, hv, one(len(hs))), sets=(ss, off, mb))
        for over in ({"gauges": recs(cls[1] + 1)},
                     {"sets": (np.zeros(cls[3] + 1, np.uint32), np.arange(cls[3] + 2, dtype=np.uint32), mb)},
                     {"histos": recs(cls[2] + 1) + (one(cls[2] + 1),)}):
            with pytest.raises(V.EngineError):  # one record over the class's cap, within max_batch_records
                e.ingest(**over)
        f = e.flush()
    # every record of the capped batch landed (the rejected ones left no trace)
    assert dict(zip(f.counter_slot.tolist(), f.counter_value.tolist())) == \
        {s: w.counter_value(s) for s in range(64) if w.touched(0, s)}
    assert dict(zip(f.gauge_slot.tolist(), f.gauge_value.tolist())) == \
        {s: w.gauge_value(s) for s in range(64) if w.touched(1, s)}
    assert f.set_estimate.tolist() == [w.set_estimate(int(s)) for s in f.set_slot]
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_quantiles, oq)
    with pytest.raises(V.EngineError):
        V.Engine(caps, max_batch_records=256, max_class_records=(300, 0, 0, 0))


@pytest.mark.parametrize("path", ["host", "device"])
def test_counter_any_sample_rate_as_go(path):
    """Counter.Sample (samplers.go:133) is defined for every float32 rate: int64(float32(1/rate))
    is MinInt64 on amd64 for NaN (which the parser lets through), 0 (+Inf) and rates whose
    reciprocal passes 2^63, and a plain truncation otherwise (rates above 1 give 0); the product
    with int64(sample) wraps.  Both ingest paths take such records and equal the oracle."""
    rng = np.random.default_rng(21)
    n, cap = 16000, 97
    slots = rng.integers(0, cap, n).astype(np.uint32)
    vals = rng.integers(-9, 10, n).astype(np.float64) + rng.choice([0.0, 0.5, 0.99], n)
    odd = np.array([np.nan, 0.0, -0.0, 1.5, 3.0, -0.25, 1e-30, np.inf, -np.inf, 0.1, 0.3], np.float32)
    rates = np.where(rng.random(n) < 0.3, rng.choice(odd, n), np.float32(1.0)).astype(np.float32)
    w = oracle.Worker(cap, 1, 1, 1)
    w.counter(slots, vals, rates)
    bufs = []
    with make_engine((cap, 1, 1, 1)) as e:
        if path == "host":
            e.ingest(counters=(slots, vals, rates))
        else:
            e.ingest_device(_device_batch(bufs, counters=(slots, vals, rates)))
        f = e.flush()
    for b in bufs:
        b.free()
    want = {s: w.counter_value(s) for s in range(cap) if w.touched(0, s)}
    assert dict(zip(f.counter_slot.tolist(), f.counter_value.tolist())) == want
