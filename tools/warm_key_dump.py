#!/usr/bin/env python3
"""Dump the C4 window's samples (arrival order) of chosen histogram slots, as bench.py generates
them, for CPU studies of the hot-key remainder (tools/tdigest_study.py strategies).
    python tools/warm_key_dump.py OUT.npz SLOT [SLOT ...]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("slots", type=int, nargs="+")
    ap.add_argument("--seed", type=int, default=0x5EED0004)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--samples", type=int, default=1_000_000_000)
    a = ap.parse_args()
    import bench
    import veneur_amd as V
    sample = min(a.samples, 1 << 24)
    counts = V.synth_key_counts(a.seed, a.keys, a.samples, sample, device=0)
    classes = bench.key_classes(a.seed, a.keys)
    thr = a.samples / (1 * 32)
    split = bench.hot_keys(counts, a.samples / sample, classes, thr, min(thr, 1 << 18), 64)
    st = V.DeviceStream(a.seed, a.keys, a.samples, 0, 1, device=0, split=split)
    d = st.to_host()
    out = {}
    for s in a.slots:
        m = d["h_slot"] == s
        out["v%d" % s], out["r%d" % s] = d["h_val"][m], d["h_rate"][m]
    np.savez(a.out, **out)
    print("dumped", {s: int((d["h_slot"] == s).sum()) for s in a.slots})


if __name__ == "__main__":
    main()
