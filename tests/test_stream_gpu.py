"""The C4 stream generated in HBM (vn_synth_device, bench.py): N ranks' shares are exactly one
global stream -- ordinary keys routed by digest % N (server.go:655), split keys dealt
round-robin by their window arrival index -- and a whole C4-shaped window (split keys included)
through the engine matches the restated Go worker on the same records."""
import numpy as np
import pytest

import veneur_amd as V
from tests.util import PCT, rank_errors, run_oracle

pytestmark = pytest.mark.gpu

SEED, KEYS, N_SAMPLES = 77, 3000, 2_000_000


def _records(st):
    """per global key: list of (class, values...) in the rank's order"""
    d = st.to_host()
    out = {}
    for c, (sk, cols) in enumerate((("c_slot", ("c_val", "c_rate")), ("g_slot", ("g_val",)),
                                    ("h_slot", ("h_val", "h_rate")), ("s_slot", ()))):
        keys = st.key_of_slot[c][d[sk]]
        vals = [d[x] for x in cols]
        if c == 3:
            vals = [d["s_bytes"].reshape(-1, 11).view("S11")[:, 0]]
        for i, k in enumerate(keys.tolist()):
            out.setdefault(k, []).append(tuple(v[i] for v in vals))
    return out, d


def test_ranks_partition_one_global_stream():
    counts = V.synth_key_counts(SEED, KEYS, N_SAMPLES, N_SAMPLES)
    assert counts.sum() == N_SAMPLES
    top = np.argsort(-counts.astype(np.int64))[:12]
    import bench
    cls = bench.key_classes(SEED, KEYS)
    split = {c: np.sort(top[cls[top] == c]).astype(np.uint32) for c in (0, 2, 3)}
    one = V.DeviceStream(SEED, KEYS, N_SAMPLES, 0, 1)
    ref, _ = _records(one)
    assert sum(len(v) for v in ref.values()) == N_SAMPLES
    assert all(len(ref.get(k, [])) == counts[k] for k in range(KEYS))
    one.free()
    N = 3
    shares = [V.DeviceStream(SEED, KEYS, N_SAMPLES, r, N, split=split) for r in range(N)]
    recs = [_records(s)[0] for s in shares]
    assert sum(s.n_records for s in shares) == N_SAMPLES
    splitset = set(int(k) for c in split for k in split[c])
    for k, rk in ref.items():
        if k in splitset:  # record j of the key on rank j % N, in order
            for r in range(N):
                assert recs[r].get(k, []) == rk[r::N], k
        else:
            owners = [r for r in range(N) if k in recs[r]]
            assert len(owners) == 1, k
            assert recs[owners[0]][k] == rk, k
    for s in shares:
        s.free()


def test_c4_window_through_engine_matches_oracle():
    """One rank, the hottest keys split (the single-GPU split path; split timers are gathered whole
    to their owner and replayed there): counters, gauges and sets bit-exact, histogram Local*
    stats exact, quantiles identical to the restated Go (the default exact mode)."""
    import bench
    counts = V.synth_key_counts(SEED, KEYS, N_SAMPLES, N_SAMPLES)
    split = bench.hot_keys(counts, 1.0, bench.key_classes(SEED, KEYS), N_SAMPLES / 128, 10000, 16,
                           split_histos=True)
    assert all(len(split[c]) for c in (0, 2, 3))
    st = V.DeviceStream(SEED, KEYS, N_SAMPLES, 0, 1, split=split)
    d = st.to_host()
    n = st.n_slots
    with V.Engine(n, percentiles=PCT, max_batch_records=max(st.counts) + 1, max_batch_member_bytes=st.counts[3] * 11 + 64,
                  split_max_records=max(st.split_counts) + 1) as e:
        for c in (0, 2, 3):
            slots = (st.split_slot0[c] + np.arange(len(split[c]))).astype(np.uint32)
            e.split_keys(c, slots, np.zeros(len(slots), np.uint32))
        e.ingest_device(st.batch)
        e.ingest_split_device(st.split)
        f = e.flush()
    w = run_oracle(d, n)
    assert dict(zip(f.counter_slot.tolist(), f.counter_value.tolist())) == \
        {s: w.counter_value(s) for s in range(n[0]) if w.touched(0, s)}
    assert dict(zip(f.gauge_slot.tolist(), f.gauge_value.tolist())) == \
        {s: w.gauge_value(s) for s in range(n[1]) if w.touched(1, s)}
    assert dict(zip(f.set_slot.tolist(), f.set_estimate.tolist())) == \
        {s: w.set_estimate(s) for s in range(n[3]) if w.touched(3, s)}
    ost = np.array([w.histo_stats(int(s)) for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_stats[:, [0, 1, 2]], ost[:, [0, 1, 2]])
    np.testing.assert_allclose(f.histo_stats[:, 3:5], ost[:, 3:5], rtol=1e-12)
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    err = rank_errors(d, f.histo_slot, f.histo_quantiles, oq)
    assert err.max() <= 1e-3, err.max()
    np.testing.assert_array_equal(f.histo_quantiles, oq)
    st.free()


def test_c4_window_tenth_scale_every_key_bit_exact():
    """The C4 window at a tenth of its size -- 100k keys, 100M samples, the bench's stream, every key
    on its owner (the default exact mode, no split) -- against the restated Go worker over every
    key of every class: counters, gauges and set estimates bit-exact, histogram min/max/weight
    exact, sums within 1e-12, every histogram key's quantiles bit-identical (the hottest timer key
    here holds ~1.9M samples: the batched replay)."""
    keys, n_samples = 100_000, 100_000_000
    st = V.DeviceStream(SEED, keys, n_samples, 0, 1)
    d = st.to_host()
    n = st.n_slots
    with V.Engine(n, percentiles=PCT, max_batch_records=max(st.counts) + 1,
                  max_batch_member_bytes=st.counts[3] * 11 + 64) as e:
        e.ingest_device(st.batch)
        f = e.flush()
    st.free()
    w = run_oracle(d, n)
    assert dict(zip(f.counter_slot.tolist(), f.counter_value.tolist())) == \
        {s: w.counter_value(s) for s in range(n[0]) if w.touched(0, s)}
    assert dict(zip(f.gauge_slot.tolist(), f.gauge_value.tolist())) == \
        {s: w.gauge_value(s) for s in range(n[1]) if w.touched(1, s)}
    assert dict(zip(f.set_slot.tolist(), f.set_estimate.tolist())) == \
        {s: w.set_estimate(s) for s in range(n[3]) if w.touched(3, s)}
    ost = np.array([w.histo_stats(int(s)) for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_stats[:, [0, 1, 2]], ost[:, [0, 1, 2]])
    np.testing.assert_allclose(f.histo_stats[:, 3:5], ost[:, 3:5], rtol=1e-12)
    oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
    np.testing.assert_array_equal(f.histo_quantiles, oq)
