"""World-size-2 (gloo, CPU) test of the pipelined flush windows (veneur_amd.dist.InTurn, bench.py
--pipeline D): D engines per rank take the windows in turn, one communicator per engine, and each
rank enters a window's split combine only in window order.

The combine here is the CPU restatement of the engine's (tests/split_protocol.py: counters by
all-reduce, sets by gathered records and the dense epochs) over one gloo subgroup per engine, so
the test checks the orchestration the GPU path relies on:
  * every collective of a communicator pairs the same window on both ranks (each combine first
    all-gathers its window id);
  * each window's combined result is the single consumer's (counter sums exact, set sketches
    bit-identical to one oracle Sketch fed the whole window);
  * ranks running at different speeds (random, rank-dependent ingest delays) never deadlock.
"""
import os
import random
import socket
import time

import numpy as np
import torch.multiprocessing as mp

import oracle
from tests import split_protocol as SP
from veneur_amd import dist as D

WINDOWS, ENGINES = 6, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _window(i):
    rng = np.random.default_rng(100 + i)
    ctr = rng.integers(-3, 40, (3, 3000)).astype(np.int64)
    u = rng.integers(0, 2**64 - 1, 400 + 300 * i, dtype=np.uint64)
    hs = u[rng.integers(0, len(u), 6000)]
    return ctr, hs


class _Sub:
    """One engine's communicator: a gloo subgroup with the Group calls split_protocol makes."""

    def __init__(self, td, pg, world, rank):
        self.td, self.pg, self.world, self.rank = td, pg, world, rank
        self.dist = self
        self.ReduceOp = td.ReduceOp

    def all_reduce(self, t, op):
        self.td.all_reduce(t, op=op, group=self.pg)

    def gather_object(self, obj):
        out = [None] * self.world
        self.td.all_gather_object(out, obj, group=self.pg)
        return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    try:
        g = D.Group(backend="gloo")
        import torch.distributed as td
        subs = [_Sub(td, td.new_group(ranks=list(range(world))), world, rank) for _ in range(ENGINES)]
        rnd = random.Random(rank * 7919)
        entered = []

        def work(k, i, turn):
            ctr, hs = _window(i)
            time.sleep(rnd.random() * 0.05)  # this rank's ingest of window i, of a varying length
            part = np.array([c[D.deal(len(c), world) == rank].sum() for c in ctr], np.int64)
            share = hs[D.deal(len(hs), world) == rank]
            with turn(i):
                entered.append(i)
                ids = subs[k].gather_object(i)  # the communicator's peers are on the same window
                c = SP.counters(subs[k], part)
                sk = SP.sets(subs[k], share, len(hs))
            return {"window": i, "engine": k, "peer_windows": ids, "counters": c.tolist(),
                    "set": (sk.sparse, sk.b, sk.estimate(),
                            sk.registers().tolist() if not sk.sparse else sorted(sk.list_codes().tolist()))}

        out = D.InTurn(ENGINES).run(WINDOWS, work)
        res = {"rank": rank, "entered": entered, "out": out}
        allres = g.gather_object(res)
        g.barrier()
        g.close()
        if rank == 0:
            q.put(allres)
    except Exception as ex:  # surface the failure in the parent
        q.put(repr(ex))
        raise


def test_pipelined_windows_two_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        allres = q.get(timeout=600)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert not isinstance(allres, str), allres
    assert all(p.exitcode == 0 for p in procs)
    for r in allres:
        assert r["entered"] == list(range(WINDOWS))
        for i, o in enumerate(r["out"]):
            assert o["window"] == i and o["engine"] == i % ENGINES
            assert o["peer_windows"] == [i] * world
            ctr, hs = _window(i)
            assert o["counters"] == ctr.sum(axis=1).tolist()
            sk = oracle.Sketch()
            for x in hs.tolist():
                sk.insert_hash(int(x))
            exp = (sk.sparse, sk.b, sk.estimate(),
                   sk.registers().tolist() if not sk.sparse else sorted(sk.list_codes().tolist()))
            assert tuple(o["set"]) == exp, i
