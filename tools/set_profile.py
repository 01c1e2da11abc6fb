#!/usr/bin/env python3
"""Where k_set_segments spends its workgroup time (GPU box; VN_SET_PROF variant build:
make -C veneur_amd variant VARIANT_FLAGS=-DVN_SET_PROF).  Ingests the set records of the C4 window
(DeviceStream, no split keys) and prints the clock64 cycles summed over workgroups per phase.
    VN_LIB=libveneur_amd_variant.so python tools/set_profile.py"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VN_LIB", "libveneur_amd_variant.so")
import veneur_amd as V  # noqa: E402
import veneur_amd._abi as A  # noqa: E402

A.lib.vn_prof_set_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
NAMES = ["setup", "sparse scan", "sparse merge", "toNormal", "dense", "write-back", "triggers", "heavy keys",
         "heavy records", "workgroups", "group merges", "group codes", "group fallbacks", "single merges", "longest workgroup",
         "its records"]


def main():
    st = V.DeviceStream(0x5EED0004, 1_000_000, 1_000_000_000, 0, 1, device=0, split=None)
    b = st.batch
    n_set = int(b.n_set)
    batch = A.Batch()
    batch.n_set = n_set
    batch.set_slot, batch.set_member_off, batch.set_member_bytes = b.set_slot, b.set_member_off, b.set_member_bytes
    caps = (1, 1, 1, max(1, st.n_slots[3]))
    with V.Engine(caps, percentiles=(0.5,), max_batch_records=n_set + 1, max_batch_member_bytes=n_set * 11 + 64) as e:
        for rep in range(3):
            e.timing_enable(True)
            buf = (C.c_ulonglong * 40)()
            A.lib.vn_prof_set_read(buf, 1)
            assert A.lib.vn_ingest(e.h, C.byref(batch)) == 0, A.lib.vn_last_error(e.h)
            e.flush_raw()
            t = e.timing()
            A.lib.vn_prof_set_read(buf, 0)
            tot = buf[9] or 1
            print("rep %d: %d set records, %d keys; k_set_small + k_set_segments %.2f ms" %
                  (rep, n_set, st.n_slots[3], t["ms_set_segments"]))
            for i, nm in enumerate(NAMES):
                v = buf[i]
                print("   %-14s %16d %s" % (nm, v, ("%5.1f%%" % (100.0 * v / tot)) if i < 6 or i == 9 else ""))
            print("   workgroup 0 (the key with the most records):",
                  {NAMES[i]: int(buf[16 + i]) for i in (0, 1, 2, 3, 4, 5, 9)})
            print("   workgroup 0's dense phase:", dict(zip(("chunks", "passes", "fill cycles", "marking cycles",
                                                             "full-path cycles", "rebases", "rebase cycles",
                                                             "chunk-top cycles"), (int(v) for v in buf[32:40]))))


if __name__ == "__main__":
    main()
