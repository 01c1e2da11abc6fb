"""CPU tests of the bench's split-list choice from the engines' hot-key detector
(bench.split_from_engine): candidates summed over the ranks, class thresholds, the cap, and the
hysteresis that keeps a split key while it stays above half the threshold."""
import numpy as np

import bench
from veneur_amd.dist import InTurn


class FakeEngine:
    def __init__(self, table):
        self.table = table  # {cls: [(slot, count)]}
        self.asked = []

    def hot_keys(self, cls, min_count, cap):
        self.asked.append((cls, min_count, cap))
        rows = sorted([r for r in self.table.get(cls, []) if r[1] >= min_count], key=lambda r: (-r[1], r[0]))[:cap]
        return (np.array([r[0] for r in rows], np.uint32), np.array([r[1] for r in rows], np.uint64))


class FakeCtrl:
    def __init__(self, world, others):
        self.world = world
        self.others = others  # the other ranks' local candidate dicts

    def gather_object(self, obj):
        return [obj] + self.others


def test_sum_over_ranks_threshold_cap_and_key_ids():
    key_of_slot = {0: np.array([100, 101, 102, 103], np.uint32), 3: np.array([200, 201], np.uint32)}
    e = FakeEngine({0: [(0, 600), (1, 400), (2, 90)], 3: [(1, 50)]})
    # rank 1 holds a share of key 101 (dealt) and its own key 150
    ctrl = FakeCtrl(2, [{0: [(101, 300), (150, 900)], 3: [(201, 60)]}])
    split = bench.split_from_engine(e, key_of_slot, {0: 500, 3: 100}, ctrl, max_split=2)
    assert split[0].tolist() == [101, 150]  # 700 and 900; 100 (600) is third, over the cap
    assert split[3].tolist() == [201]       # 50 + 60 > 100
    assert split[2].tolist() == []
    # each rank asks for its share of half the threshold
    assert (0, 500 // 4 + 1, 32) in e.asked


def test_hysteresis_keeps_a_split_key_above_half_the_threshold():
    key_of_slot = {0: np.array([10, 11], np.uint32)}
    e = FakeEngine({0: [(0, 300), (1, 700)]})
    ctrl = FakeCtrl(1, [])
    fresh = bench.split_from_engine(e, key_of_slot, {0: 500}, ctrl, max_split=8)
    assert fresh[0].tolist() == [11]
    kept = bench.split_from_engine(e, key_of_slot, {0: 500}, ctrl, max_split=8, keep={0: np.array([10, 11])})
    assert kept[0].tolist() == [10, 11]
    e2 = FakeEngine({0: [(0, 200), (1, 700)]})
    assert bench.split_from_engine(e2, key_of_slot, {0: 500}, ctrl, max_split=8,
                                   keep={0: np.array([10, 11])})[0].tolist() == [11]


def test_windows_in_turn_flush_in_window_order_and_fail_without_hanging():
    import random
    import threading
    import time

    import pytest

    order, per_engine, lock = [], {}, threading.Lock()

    def work(k, i, turn):
        time.sleep(random.random() * 0.01)  # ingest of a varying length
        with lock:
            per_engine.setdefault(k, []).append(i)
        with turn(i):
            with lock:
                order.append(i)
        return (k, i)

    for D in (1, 2, 3):
        order.clear()
        per_engine.clear()
        out = InTurn(D).run(10, work)
        assert order == list(range(10))
        assert out == [(i % D, i) for i in range(10)]
        assert all(v == sorted(v) and all(i % D == k for i in v) for k, v in per_engine.items())

    def bad(k, i, turn):
        if i == 4:
            raise RuntimeError("window 4")
        with turn(i):
            pass
        return i

    t0 = time.time()
    with pytest.raises(RuntimeError, match="window 4"):
        InTurn(2).run(10, bad)
    assert time.time() - t0 < 5
