"""GPU tests of the engine's hot-key detector (vn_hot_detect / vn_hot_keys, hotkeys.hip).

The reference routes every record of a key to one worker (server.go:655); splitting a hot key
over the ranks is this build's addition, so the engine picks the next window's split list itself
from the window it saw.  Checked against numpy counts of the same records: exact at stride 1, the
fixed strided sample otherwise; split records count for their slots through the split list."""
import numpy as np
import pytest

import veneur_amd as V

pytestmark = pytest.mark.gpu


def zipf_slots(rng, n, nk):
    return np.minimum(rng.zipf(1.3, n) - 1, nk - 1).astype(np.uint32)


def expected(slots_per_call, stride, min_count, cap):
    cnt = {}
    for s in slots_per_call:
        for x in s[::stride].tolist():
            cnt[x] = cnt.get(x, 0) + 1
    items = [(c * stride, k) for k, c in cnt.items() if c * stride >= min_count]
    items.sort(key=lambda t: (-t[0], t[1]))
    items = items[:cap]
    return [k for _, k in items], [c for c, _ in items]


@pytest.mark.parametrize("stride", [1, 3])
def test_hot_keys_match_numpy_counts(stride):
    rng = np.random.default_rng(40 + stride)
    nk = 500
    calls = []
    with V.Engine((nk, 1, nk, nk), max_batch_records=1 << 16) as e:
        e.hot_detect(stride)
        for _ in range(3):
            n = 20000
            cs, hs, ss = zipf_slots(rng, n, nk), zipf_slots(rng, n, nk), zipf_slots(rng, n, nk)
            e.ingest(counters=(cs, np.ones(n), np.ones(n, np.float32)),
                     histos=(hs, rng.random(n), np.ones(n, np.float32)),
                     set_hashes=(ss, rng.integers(0, 2**63, n, dtype=np.uint64)))
            calls.append((cs, hs, ss))
        e.flush()
        for cls, pos in ((0, 0), (2, 1), (3, 2)):
            for thr, cap in ((500, 64), (1, 10), (50, 1000)):
                slots, counts = e.hot_keys(cls, thr, cap)
                ks, cs_ = expected([c[pos] for c in calls], stride, thr, cap)
                assert slots.tolist() == ks, (cls, thr, cap)
                assert counts.tolist() == cs_, (cls, thr, cap)
        with pytest.raises(V.EngineError):
            e.hot_keys(1, 1)  # gauges cannot be split
        # the next window starts from zero: an empty window reports nothing
        e.flush()
        assert e.hot_keys(0, 1)[0].tolist() == []


def test_hot_keys_count_split_records_through_the_split_list():
    rng = np.random.default_rng(44)
    split_slots = np.array([7, 3], np.uint32)
    with V.Engine((1, 1, 16, 16), max_batch_records=1 << 16, split_max_records=1 << 16) as e:
        e.hot_detect(1)
        e.split_keys(2, split_slots, np.zeros(2, np.uint32))
        keys = rng.integers(0, 2, 5000).astype(np.uint32)
        e.ingest_split(histos=(keys, rng.random(5000), np.ones(5000, np.float32)))
        direct = np.setdiff1d(np.arange(16, dtype=np.uint32), split_slots)  # (a split slot takes no direct records)
        hs = direct[rng.integers(0, len(direct), 3000)]
        e.ingest(histos=(hs, rng.random(3000), np.ones(3000, np.float32)))
        e.flush()
        slots, counts = e.hot_keys(2, 1, 16)
        ks, cs = expected([hs, split_slots[keys]], 1, 1, 16)
        assert slots.tolist() == ks and counts.tolist() == cs
        # detection off: the following windows report nothing new
        e.hot_detect(0)
        e.ingest(histos=(hs, rng.random(3000), np.ones(3000, np.float32)))
        e.flush()
        assert e.hot_keys(2, 1)[0].tolist() == []
