#!/usr/bin/env python3
"""Debug aid (GPU box): the same prefix ingested R times into fresh engines; prints the centroid
count after export each time (a race would show as varying results)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import veneur_amd as V
    d = np.load(sys.argv[1])
    n = int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    v, r = d["v"][:n], d["r"][:n]
    slot = np.zeros(n, np.uint32)
    res = []
    for _ in range(reps):
        with V.Engine((1, 1, 1, 1), percentiles=(0.5,), max_batch_records=n + 1) as e:
            e.ingest(histos=(slot, v, r))
            m0, _, _ = e.read_histo(0)
            e.export_histos(np.zeros(1, np.uint32))
            m, w, _ = e.read_histo(0)
            e.flush()
        res.append((len(m0), len(m), float(m[-1]), float(w[-1])))
    print(os.environ.get("VN_LIB", "default"), n, res, flush=True)


if __name__ == "__main__":
    main()
