#!/usr/bin/env python3
"""Rank error of a t-digest key split across N GPUs against one consumer.

The single-GPU hot-key scheme replays a key's first P window samples exactly,
then merges geometric pieces [b_i, b_{i+1}) (b_{i+1} = b_i + b_i*g/100) one mergeAllTemps each.
A split key's samples are dealt round-robin over N ranks (window index j -> rank j % N), so
no rank holds a whole piece.  The owner instead merges, per piece, the union of every rank's
*micro-centroids* of its share of that piece: the share sorted and compressed on its own rank
by one mergeAllTemps at a finer compression delta_hi.  This study measures what that costs
against the reference's 42-sample incremental digest (oracle, Add() in order), next to the
single-GPU scheme on the same samples.  CPU only; the oracle is the reference.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from tools.tdigest_study import PCT, quantiles, rank_err, sample  # noqa: E402


def pieces(n, P, g):
    b = [P]
    while b[-1] < n:
        b.append(b[-1] + max(1, b[-1] * g // 100))
    b[-1] = min(b[-1], n)
    return list(zip(b[:-1], b[1:]))


def single(v, w, P, g):
    td = oracle.MergingDigest(100.0)
    td.add_many(v[:P], w[:P])
    for a, b in pieces(len(v), P, g):
        td.add_batch(v[a:b], w[a:b])
    return quantiles(td)


def split(v, w, P, g, N, dhi):
    td = oracle.MergingDigest(100.0)
    td.add_many(v[:P], w[:P])
    for a, b in pieces(len(v), P, g):
        ms, ws = [], []
        for r in range(N):
            j0 = a + ((r - a) % N)
            sv, sw = v[j0:b:N], w[j0:b:N]
            if len(sv) == 0:
                continue
            md = oracle.MergingDigest(float(dhi))
            md.add_batch(sv, sw)
            m, cw = md.centroids()
            ms.append(m)
            ws.append(cw)
        td.add_batch(np.concatenate(ms), np.concatenate(ws))
    return quantiles(td)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="50000,200000,1000000,3000000")
    ap.add_argument("--seeds", type=int, default=4)
    ap.add_argument("--N", default="2,8")
    ap.add_argument("--dhi", default="200,500,1000")
    ap.add_argument("--P", type=int, default=4096)
    ap.add_argument("--g", type=int, default=25)
    a = ap.parse_args()
    for n in [int(x) for x in a.sizes.split(",")]:
        worst = {}
        for sd in range(a.seeds):
            rng = np.random.default_rng(7000 * n + sd)
            v, w = sample(n, rng)
            go = oracle.MergingDigest(100.0)
            go.add_many(v, w)
            qg = quantiles(go)
            k = ("single", 0, 0)
            worst[k] = np.maximum(worst.get(k, 0), rank_err(v, w, single(v, w, a.P, a.g), qg))
            for N in [int(x) for x in a.N.split(",")]:
                for dhi in [int(x) for x in a.dhi.split(",")]:
                    k = ("split", N, dhi)
                    worst[k] = np.maximum(worst.get(k, 0), rank_err(v, w, split(v, w, a.P, a.g, N, dhi), qg))
        for (m, N, dhi), err in sorted(worst.items()):
            print("n=%8d %-6s N=%d dhi=%4d max rank err p50 %.2e p90 %.2e p99 %.2e p99.9 %.2e" %
                  ((n, m, N, dhi) + tuple(err)), flush=True)


if __name__ == "__main__":
    main()
