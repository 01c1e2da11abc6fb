#!/usr/bin/env python3
"""The hot-key remainder scheme on real C4 keys (dumped by tools/warm_key_dump.py): rank error of
the CPU restatement of the engine's scheme against the restated Go digest for several exact
prefixes E and piece growths g, and each side's distance from the key's exact quantile |F(q) - p|.
    python tools/remainder_accuracy.py gpurun_out/warm_keys.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from tools.tdigest_study import PCT, quantiles, rank_err, strategy  # noqa: E402


def main(path):
    d = np.load(path)
    for s in sorted(int(k[1:]) for k in d.files if k.startswith("v")):
        v, r = d["v%d" % s], d["r%d" % s]
        w = (np.float32(1.0) / r.astype(np.float32)).astype(np.float64)
        go = oracle.MergingDigest(100.0)
        go.add_many(v, w)
        qg = quantiles(go)
        o = np.argsort(v, kind="stable")
        sv, cw = v[o], np.cumsum(w[o])
        F = lambda q: cw[np.searchsorted(sv, q, side="right") - 1] / cw[-1] if np.searchsorted(sv, q, side="right") else 0.0
        line = ["slot %d n=%d" % (s, len(v))]
        for E, g in ((32768, 25), (4096, 25), (32768, 10)):
            q = strategy(v, w, E, "geom", g)
            line.append("E=%d g=%d rank err %s" % (E, g, np.round(rank_err(v, w, q, qg), 6).tolist()))
        eng = strategy(v, w, 32768 if len(v) <= 4 * 32768 else 4096, "geom", 25)
        line.append("|F-p| go %s engine %s" % (np.round([abs(F(a) - p) for a, p in zip(qg, PCT)], 6).tolist(),
                                              np.round([abs(F(a) - p) for a, p in zip(eng, PCT)], 6).tolist()))
        print("\n  ".join(line), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
