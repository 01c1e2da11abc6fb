"""Probe (not product): the [3] case of tests/test_batch_replay_gpu.py ingested call by call; after
each call every long key's main centroids (vn_read_histo: pending temps not merged) against the
restated Go digest fed the same prefix of that key's samples (oracle main_centroids).  Prints the
first call and key whose state differs, and whether it holds NaN."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import oracle  # noqa: E402
import veneur_amd as V  # noqa: E402
from tests.test_batch_replay_gpu import PCT, _stream  # noqa: E402

batches = int(sys.argv[1]) if len(sys.argv) > 1 else 3
kinds = ["lognormal", "falling", "rising", "ints", "seven", "heavy"]
slot, val, rate, nk = _stream(kinds, 300_000, 11 + batches)
wts = (np.float32(1.0) / rate).astype(np.float64)
cuts = np.linspace(0, len(slot), batches + 1).astype(int)
with V.Engine((1, 1, nk, 1), percentiles=PCT, max_batch_records=len(slot) + 1) as e:
    for c, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        e.ingest(histos=(slot[a:b], val[a:b], rate[a:b]))
        for k, kind in enumerate(kinds):
            sel = slot[:b] == k
            td = oracle.MergingDigest(100.0)
            td.add_many(val[:b][sel], wts[:b][sel])
            om, ow = td.main_centroids()
            gm, gw, st = e.read_histo(k)
            same = len(om) == len(gm) and np.array_equal(om, gm) and np.array_equal(ow, gw)
            if not same:
                n = min(len(om), len(gm))
                bad = np.nonzero((om[:n] != gm[:n]) | (ow[:n] != gw[:n]))[0]
                i = int(bad[0]) if len(bad) else n
                print("call %d key %d %s: %d centroids (gpu) vs %d; first diff %d: gpu %r %r ref %r %r; nan %s; mainW %r vs %r"
                      % (c, k, kind, len(gm), len(om), i, gm[i:i + 2], gw[i:i + 2], om[i:i + 2], ow[i:i + 2],
                         bool(np.isnan(gm).any() or np.isnan(gw).any()), st[7], float(np.sum(ow))), flush=True)
            else:
                print("call %d key %d %s: same (%d centroids)" % (c, k, kind, len(gm)), flush=True)
