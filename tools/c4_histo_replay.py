#!/usr/bin/env python3
"""The C4 window's timers alone (DeviceStream, histogram records only) through one engine:
ms of ingest + flush, and with the profiling build (VN_LIB=libveneur_amd_prof.so) the merge
phase cycles of the four-wave replay's block 0 (the longest key)."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import veneur_amd as V  # noqa: E402
import veneur_amd._abi as A  # noqa: E402


def main():
    samples = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    st = V.DeviceStream(0x5EED0004, 1_000_000, samples, 0, 1)
    b = A.Batch()
    src = st.batch
    b.n_histo, b.histo_slot, b.histo_value, b.histo_rate = src.n_histo, src.histo_slot, src.histo_value, src.histo_rate
    prof = hasattr(A.lib, "vn_prof_exact_read")
    if prof:
        A.lib.vn_prof_exact_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    sl = np.zeros(int(src.n_histo), np.uint32)
    A.lib.vn_copy_to_host(0, sl.ctypes.data_as(C.c_void_p), C.c_void_p(src.histo_slot), sl.nbytes)
    cnt = np.bincount(sl)
    top = np.sort(cnt)[::-1]
    print({"top_counts": top[:8].tolist(), "keys_ge_8192": int((cnt >= 8192).sum()),
           "samples_in_keys_ge_8192": int(cnt[cnt >= 8192].sum())}, flush=True)
    del sl
    with V.Engine((1, 1, st.n_slots[2], 1), percentiles=(0.5, 0.9, 0.99, 0.999), max_batch_records=int(src.n_histo) + 1) as e:
        for rep in range(3):
            buf = (C.c_ulonglong * 16)()
            if prof:
                A.lib.vn_prof_exact_read(buf, 1)
            A.lib.vn_device_synchronize(0)
            t0 = time.perf_counter()
            e.ingest_device(b)
            e.flush_raw()
            A.lib.vn_device_synchronize(0)
            ms = (time.perf_counter() - t0) * 1e3
            out = {"rep": rep, "histo_records": int(src.n_histo), "ms": round(ms, 2)}
            if prof:
                A.lib.vn_prof_exact_read(buf, 1)
                p = list(buf)
                mg = max(1, p[5])
                out.update({"merges_block0": p[5], "cyc_A": round(p[1] / mg), "cyc_B": round(p[2] / mg),
                            "cyc_C": round(p[3] / mg), "cyc_D": round(p[4] / mg), "walked": p[12]})
            print(out, flush=True)
    st.free()


if __name__ == "__main__":
    main()
