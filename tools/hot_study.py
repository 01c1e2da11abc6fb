#!/usr/bin/env python3
"""Tail of the hot-key t-digest scheme's rank error over a C4-like population of keys.

The engine replays a key's first samples exactly (MergingDigest.Add, bit-identical) and merges
the rest in geometric pieces: cold keys (<= E samples) are exact; warm keys
(E < n <= W*E) replay E samples then pieces; hot keys replay P samples then pieces growing by g%.
This study draws key sizes like C4's Zipf tail above E and reports the distribution of
|F(q_scheme) - F(q_go)| over many keys for variants of (P, g, W, piece cap), so the tail --
not just a few seeds -- is what a setting is judged by.  CPU only (oracle = the reference).
"""
import argparse
import os
import sys
from multiprocessing import Pool

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from tools.tdigest_study import PCT, quantiles, rank_err, sample  # noqa: E402


def scheme(v, w, E, P, g, W, cap):
    n = len(v)
    td = oracle.MergingDigest(100.0)
    if n <= E:
        td.add_many(v, w)
        return quantiles(td)
    pre = E if n <= W * E else P
    td.add_many(v[:pre], w[:pre])
    b = pre
    bounds = []
    x = P
    while x < n:
        nx = x + max(1, x * g // 100)
        if cap:
            nx = min(nx, x + cap)
        bounds.append((x, nx))
        x = nx
    # pieces cut at the window positions b_i (from P), starting where the exact part ended
    for lo, hi in bounds:
        lo, hi = max(lo, pre), min(hi, n)
        if hi <= lo:
            continue
        td.add_batch(v[lo:hi], w[lo:hi])
    return quantiles(td)


def one(args):
    n, seed, variants = args
    rng = np.random.default_rng(seed)
    v, w = sample(n, rng)
    go = oracle.MergingDigest(100.0)
    go.add_many(v, w)
    qg = quantiles(go)
    return n, [rank_err(v, w, scheme(v, w, *var), qg) for var in variants]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=400)
    ap.add_argument("--max-n", type=int, default=3_000_000)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--variants", default="32768,4096,25,4,0;32768,16384,25,4,0;32768,4096,10,4,0;"
                                           "32768,4096,25,4,65536;32768,32768,25,1,0")
    a = ap.parse_args()
    variants = [tuple(int(x) for x in s.split(",")) for s in a.variants.split(";")]
    rng = np.random.default_rng(12345)
    # Zipf(1) sizes above 32768: n_k ~ C / k  ->  k uniform in log space
    lo, hi = np.log(32769), np.log(a.max_n)
    sizes = np.exp(rng.uniform(lo, hi, a.keys)).astype(int)
    sizes = np.concatenate([sizes, rng.integers(32769, 140000, a.keys // 2)])
    jobs = [(int(n), 1000 + i, variants) for i, n in enumerate(sizes)]
    with Pool(a.procs) as p:
        res = p.map(one, jobs, chunksize=4)
    for vi, var in enumerate(variants):
        errs = np.array([r[1][vi] for r in res])
        worst = errs.max(axis=1)
        print("E,P,g,W,cap=%s  keys %d  max %s  p99-of-keys %.2e  frac>1e-3 %.3f" % (
            var, len(res), np.round(errs.max(axis=0), 5).tolist(), np.quantile(worst, 0.99), np.mean(worst > 1e-3)),
            flush=True)


if __name__ == "__main__":
    main()
