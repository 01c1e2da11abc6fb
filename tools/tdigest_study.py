#!/usr/bin/env python3
"""How far does a batch merge drift from MergingDigest's 42-sample incremental merge?

For keys of n samples (lognormal values, veneur's float32 1/rate weights) this compares
quantiles of the Go-exact digest (oracle, Add() in order) with the engine's strategies:
  exact E, then one mergeAllTemps of the rest        ("oneshot")
  exact E, then chunks of C samples, one merge each  ("chunk C")
  exact E, then geometric chunks of P% of the samples so far ("geom:P")
Rank error = |F(q_strategy) - F(q_go)| with F the key's exact weighted empirical CDF.
CPU only; the oracle is the reference here.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402

PCT = (0.5, 0.9, 0.99, 0.999)


def sample(n, rng):
    v = np.exp(rng.normal(3.912023005428146, 1.0, n))
    u = rng.random(n)
    r = np.where(u < 0.05, np.float32(0.1), np.where(u < 0.10, np.float32(0.5), np.float32(1.0))).astype(np.float32)
    w = (np.float32(1.0) / r).astype(np.float64)
    return v, w


def quantiles(td):
    return np.array([td.quantile(p) for p in PCT])


def rank_err(v, w, qa, qb):
    o = np.argsort(v, kind="stable")
    sv, cw = v[o], np.cumsum(w[o])
    tot = cw[-1]
    F = lambda q: (cw[np.searchsorted(sv, q, side="right") - 1] / tot) if np.searchsorted(sv, q, side="right") else 0.0
    return np.array([abs(F(a) - F(b)) for a, b in zip(qa, qb)])


def strategy(v, w, E, mode, C=0):
    td = oracle.MergingDigest(100.0)
    e = min(E, len(v))
    td.add_many(v[:e], w[:e])
    i = e
    while i < len(v):
        if mode == "oneshot":
            j = len(v)
        elif mode == "chunk":
            j = min(len(v), i + C)
        else:  # geom: chunk = C/100 of the samples so far (C=100: doubling)
            j = min(len(v), i + max(1, (i * (C or 100)) // 100))
        td.add_batch(v[i:j], w[i:j])
        i = j
    return quantiles(td)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="20000,33000,40000,50000,70000,100000,200000,500000,1000000")
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--E", default="32768")
    ap.add_argument("--modes", default="oneshot,geom,chunk:4096,chunk:42000")
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    Es = [int(x) for x in a.E.split(",")]
    modes = a.modes.split(",")
    for n in sizes:
        worst = {}
        for sd in range(a.seeds):
            rng = np.random.default_rng(1000 * n + sd)
            v, w = sample(n, rng)
            go = oracle.MergingDigest(100.0)
            go.add_many(v, w)
            qg = quantiles(go)
            for E in Es:
                for m in modes:
                    name, _, c = m.partition(":")
                    q = strategy(v, w, E, name, int(c or 0))
                    err = rank_err(v, w, q, qg)
                    k = (E, m)
                    worst[k] = np.maximum(worst.get(k, 0), err)
        for (E, m), err in sorted(worst.items()):
            print("n=%8d E=%6d %-12s max rank err p50 %.2e p90 %.2e p99 %.2e p99.9 %.2e" %
                  ((n, E, m) + tuple(err)), flush=True)


if __name__ == "__main__":
    main()
