#!/usr/bin/env python3
"""Debug aid (GPU box): the smallest prefix of a key's sample stream whose digest differs from the
restated Go digest.  Each probe ingests the first N samples into a fresh engine and compares the
GobEncode of the key (pending temps merged, as Export does) with the oracle's.

  VN_LIB=libveneur_amd.so python tools/debug_rising.py --kind rising --n 300000
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def stream(kind, n, seed):
    from tests.test_batch_replay_gpu import _key
    return _key(kind, n, np.random.default_rng(seed))


def digest_state(gob):
    import oracle
    t = oracle.MergingDigest(100.0)
    t.gob_decode(gob)
    return t.centroids()


def probe(V, oracle, v, r, n):
    slot = np.zeros(n, np.uint32)
    w = oracle.Worker(1, 1, 1, 1)
    w.histo(slot, v[:n], r[:n])
    with V.Engine((1, 1, 1, 1), percentiles=(0.5,), max_batch_records=n + 1) as e:
        e.ingest(histos=(slot, v[:n], r[:n]))
        g = e.export_histos(np.zeros(1, np.uint32))[0]
        e.flush()
    return g == w.histo_gob(0), g, w.histo_gob(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="rising")
    ap.add_argument("--n", type=int, default=300_000)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    import oracle
    import veneur_amd as V
    v, r = stream(a.kind, a.n, a.seed)
    ok, _, _ = probe(V, oracle, v, r, a.n)
    print("full", a.n, "ok" if ok else "DIFFERS", flush=True)
    if ok:
        return
    lo, hi = 1, a.n  # prefix lo is fine, hi differs
    while hi - lo > 1:
        md = (lo + hi) // 2
        if probe(V, oracle, v, r, md)[0]:
            lo = md
        else:
            hi = md
    _, g, e = probe(V, oracle, v, r, hi)
    (mg, wg), (me, we) = digest_state(g), digest_state(e)
    print("smallest differing prefix", hi, "(largest equal", lo, ")", flush=True)
    print("engine centroids", len(mg), "oracle", len(me))
    n = min(len(mg), len(me))
    bad = np.nonzero((mg[:n] != me[:n]) | (wg[:n] != we[:n]))[0]
    i0 = int(bad[0]) if len(bad) else n
    for i in range(max(0, i0 - 2), min(max(len(mg), len(me)), i0 + 6)):
        a_ = (mg[i], wg[i]) if i < len(mg) else None
        b_ = (me[i], we[i]) if i < len(me) else None
        print(i, a_, b_)
    # the state before the failing merge and the merge's temps, for a CPU replay
    np.savez("gpurun_out/debug_%s.npz" % a.kind, v=v[:hi], r=r[:hi], hi=hi, lo=lo)


if __name__ == "__main__":
    main()
