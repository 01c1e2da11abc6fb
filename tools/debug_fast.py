#!/usr/bin/env python3
"""Debug helper: one key of n samples in one batch (the four-wave long replay when n >= 8192):
its main centroids against the oracle's after the merged prefix of the same Adds, and the flush
quantiles against the oracle's Quantile; prints the first differing centroid."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
import veneur_amd as V  # noqa: E402

PCT = (0.5, 0.9, 0.99, 0.999)
rng = np.random.default_rng(3)
for n in [int(a) for a in sys.argv[1:]] or [5000, 8400, 8401, 8442, 8443, 9000, 12000, 30000]:
    v = rng.lognormal(np.log(50.0), 1.0, n)
    r = np.ones(n, np.float32)
    with V.Engine((1, 1, 1, 1), percentiles=PCT, max_batch_records=1 << 16) as e:
        e.ingest(histos=(np.zeros(n, np.uint32), v, r))
        m, w, st = e.read_histo(0)
        e.quantile(np.zeros(1, np.uint32), [0.5])  # adopts the flush-ready digest (Quantile's merge)
        fm, fw, _ = e.read_histo(0)
        f = e.flush()
    merged = 42 * ((n - 1) // 42)
    t = oracle.MergingDigest(100.0)
    t.add_many(v[:merged], np.ones(merged))
    om, ow = t.centroids()
    same = len(m) == len(om) and np.array_equal(m, om) and np.array_equal(w, ow)
    first = -1
    if not same:
        k = min(len(m), len(om))
        d = np.nonzero((m[:k] != om[:k]) | (w[:k] != ow[:k]))[0]
        first = int(d[0]) if len(d) else k
    t2 = oracle.MergingDigest(100.0)
    t2.add_many(v, np.ones(n))
    oq = [t2.quantile(p) for p in PCT]
    tm, tw = t2.centroids()
    fs = len(fm) == len(tm) and np.array_equal(fm, tm) and np.array_equal(fw, tw)
    if not fs:
        k = min(len(fm), len(tm))
        d = np.nonzero((fm[:k] != tm[:k]) | (fw[:k] != tw[:k]))[0]
        fd = int(d[0]) if len(d) else k
        print("   flush-ready digest differs: n", len(fm), len(tm), "first", fd, "of", k, "eng",
              fm[fd - 1:fd + 3].tolist(), fw[fd - 1:fd + 3].tolist(), "ref", tm[fd - 1:fd + 3].tolist(),
              tw[fd - 1:fd + 3].tolist(), "last pending", v[merged:].max() if n > merged else None, flush=True)
    print("n", n, "ncent", len(m), len(om), "main_same", same, "first_diff", first,
          "weights", float(w.sum()), float(ow.sum()), "q_same", bool(np.array_equal(f.histo_quantiles[0], oq)),
          f.histo_quantiles[0].tolist(), oq, flush=True)
    if first >= 0:
        print("   eng", m[first:first + 3].tolist(), w[first:first + 3].tolist(), "ref", om[first:first + 3].tolist(),
              ow[first:first + 3].tolist(), flush=True)

if os.environ.get("VN_LIB", "").endswith("variant.so"):
    import ctypes as C
    import veneur_amd._abi as A
    if hasattr(A.lib, "vn_fast_dbg_read"):
        buf = (C.c_ulonglong * 64)()
        A.lib.vn_fast_dbg_read(buf)
        b = list(buf)
        f64 = lambda u: float(np.array([u], np.uint64).view(np.float64)[0])
        print("dbg hit", b[0], "m", b[1], "np", b[2], "e", b[3], "fast_flag", b[4], "nonmono", b[5], "T", f64(b[6]),
              "kv", f64(b[7]))
        print(" K[e-5..e+2]", [f64(u) for u in b[8:16]])
        print(" ref flags", b[16:24], "w", [f64(u) for u in b[24:32]])
        print(" prefix check hit", b[32], "np", b[33], "nm", b[34], "sp[np]", f64(b[35]), "tempW", f64(b[36]),
              "mp[nm]", f64(b[37]), "mainW", f64(b[38]), "sp0", f64(b[39]))
