"""Pipelined flush windows over two communicators per rank (bench.py --pipeline 2 at N > 1), on ONE
GPU: two in-process groups of N = 2 (vn_comm_init_local), engine k of rank r on group k.  Each
rank runs veneur_amd.dist.InTurn over its two engines -- window i on engine i % 2, its split
combine entered in window order, its flush outside the turn -- in host threads of its own, so the
two groups' exchanges and the engines' replays interleave as they do across GPUs.

Every window's owner results are compared with ONE consumer of that window's whole stream
(oracle): split counters exact, split set estimates exact, split timers bit-identical quantiles
(the default exact mode gathers a split timer's records to its owner in window order).
"""
import threading

import numpy as np
import pytest

import oracle
import veneur_amd as V
from veneur_amd.dist import InTurn, deal
from veneur_amd.engine import Comm
from tests.util import PCT

pytestmark = pytest.mark.gpu

N, ENGINES, WINDOWS = 2, 2, 6
CAP = (4, 1, 4, 4)


def _window(i):
    rng = np.random.default_rng(500 + i)
    c = rng.integers(-5, 60, (3, 4000)).astype(np.float64)
    h = [rng.lognormal(3.0 + 0.1 * i, 1.0, n) for n in (30_000 + 1000 * i, 700)]
    u = rng.integers(0, 2**63, 3000 + 2000 * i, dtype=np.uint64) * np.uint64(2)
    s = [u[rng.integers(0, len(u), 40_000)], u[:50]]
    return c, h, s


def test_two_groups_pipelined_windows_match_single_consumer():
    groups = [Comm.local(N) for _ in range(ENGINES)]
    eng = [[V.Engine(CAP, percentiles=PCT, max_batch_records=1 << 16, split_max_records=1 << 17)
            for _ in range(ENGINES)] for _ in range(N)]
    owners = {0: np.array([0, 1, 1], np.uint32), 2: np.array([1, 0], np.uint32), 3: np.array([1, 0], np.uint32)}
    results = [[None] * WINDOWS for _ in range(N)]
    errs = []
    try:
        for r in range(N):
            for k in range(ENGINES):
                eng[r][k].set_comm(groups[k][r])

        def work_of(r):
            def work(k, i, turn):
                e = eng[r][k]
                c, h, s = _window(i)
                e.split_keys(0, np.arange(3, dtype=np.uint32), owners[0])
                e.split_keys(2, np.arange(2, dtype=np.uint32), owners[2])
                e.split_keys(3, np.arange(2, dtype=np.uint32), owners[3])
                for key in range(3):
                    m = deal(c.shape[1], N) == r
                    e.ingest(counters=(np.full(int(m.sum()), key, np.uint32), c[key][m],
                                       np.ones(int(m.sum()), np.float32)))
                hk = np.concatenate([np.full(len(v), key, np.uint32)[deal(len(v), N) == r] for key, v in enumerate(h)])
                hv = np.concatenate([v[deal(len(v), N) == r] for v in h])
                sk = np.concatenate([np.full(len(x), key, np.uint32)[deal(len(x), N) == r] for key, x in enumerate(s)])
                sh = np.concatenate([x[deal(len(x), N) == r] for x in s])
                e.ingest_split(histos=(hk, hv, np.ones(len(hk), np.float32)), set_hashes=(sk, sh))
                with turn(i):
                    e.split_combine()
                return e.flush()
            return work

        def rank_main(r):
            try:
                results[r] = InTurn(ENGINES).run(WINDOWS, work_of(r))
            except Exception as ex:  # noqa: BLE001
                errs.append(ex)

        th = [threading.Thread(target=rank_main, args=(r,)) for r in range(N)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=600)
        assert not any(t.is_alive() for t in th), "pipelined windows did not finish"
        assert not errs, errs
    finally:
        for row in eng:
            for e in row:
                e.close()
        for g in groups:
            for c in g:
                c.close()

    for i in range(WINDOWS):
        c, h, s = _window(i)
        w = oracle.Worker(3, 1, 2, 2)
        w.counter(np.repeat(np.arange(3, dtype=np.uint32), c.shape[1]), c.ravel(), np.ones(c.size, np.float32))
        for key, v in enumerate(h):
            w.histo(np.full(len(v), key, np.uint32), v, np.ones(len(v), np.float32))
        for key, x in enumerate(s):
            w.set_hashed(np.full(len(x), key, np.uint32), x)
        for r in range(N):
            f = results[r][i]
            got_c = dict(zip(f.counter_slot.tolist(), f.counter_value.tolist()))
            assert got_c == {k: w.counter_value(k) for k in range(3) if owners[0][k] == r}, (i, r)
            got_s = dict(zip(f.set_slot.tolist(), f.set_estimate.tolist()))
            assert got_s == {k: w.set_estimate(k) for k in range(2) if owners[3][k] == r}, (i, r)
            mine = [k for k in range(2) if owners[2][k] == r]
            assert f.histo_slot.tolist() == mine, (i, r)
            for j, k in enumerate(mine):
                np.testing.assert_array_equal(f.histo_quantiles[j], [w.histo_quantile(k, p) for p in PCT])
