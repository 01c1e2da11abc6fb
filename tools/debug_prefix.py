#!/usr/bin/env python3
"""Debug aid (GPU box): the engine's unmerged main list after ingesting the first N samples of a
debug_rising stream (read_histo), and its export, saved for a CPU replay of the final merge."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import veneur_amd as V
    d = np.load(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else int(d["hi"])
    v, r = d["v"][:n], d["r"][:n]
    slot = np.zeros(n, np.uint32)
    out = {}
    for mode, thr in (("exact", 0),):
        with V.Engine((1, 1, 1, 1), percentiles=(0.5,), max_batch_records=n + 1, exact_threshold=thr) as e:
            e.ingest(histos=(slot, v, r))
            m, w, st = e.read_histo(0)
            g = e.export_histos(np.zeros(1, np.uint32))[0]
            m2, w2, st2 = e.read_histo(0)
            e.flush()
        out[mode + "_m"], out[mode + "_w"], out[mode + "_st"] = m, w, st
        out[mode + "_m2"], out[mode + "_w2"] = m2, w2
        out[mode + "_gob"] = np.frombuffer(g, np.uint8)
    np.savez("gpurun_out/debug_prefix_%d.npz" % n, **out)
    print("saved", n, len(m), len(m2), flush=True)


if __name__ == "__main__":
    main()
