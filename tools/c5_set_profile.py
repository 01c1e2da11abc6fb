#!/usr/bin/env python3
"""Where C5's set import (k_set_merge) spends its workgroup time (GPU box; VN_SET_PROF variant:
make -C veneur_amd variant VARIANT_FLAGS=-DVN_SET_PROF).  Runs the C5 leg (bench.py --c5-only:
its untimed, timed, phase and timing windows) and prints the clock64 cycles per payload kind,
summed over workgroups and all windows.
    VN_LIB=libveneur_amd_variant.so python tools/c5_set_profile.py"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("VN_LIB", "libveneur_amd_variant.so")
import bench  # noqa: E402
import veneur_amd._abi as A  # noqa: E402

NAMES = {0: "workgroups", 1: "sparse <- sparse", 2: "  payloads", 3: "dense <- runs of sparse", 4: "  runs",
         5: "  payloads", 6: "dense <- sparse, one at a time", 7: "  payloads", 8: "dense payloads", 9: "  payloads",
         10: "toNormal", 11: "payloads in all", 12: "  sparse: tmpSet load + sort", 13: "  sparse: list decode",
         14: "  sparse: unique + union + lookup", 15: "  sparse: mergeSparse triggers",
         16: "    trigger: tmpSet union + lookups", 17: "    trigger: list union", 18: "  sparse: tmpSet union (no trigger)"}


def main():
    A.lib.vn_prof_import_set_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 24)()
    A.lib.vn_prof_import_set_read(buf, 1)
    sys.argv = ["bench.py", "--c5-only"]
    bench.main()
    A.lib.vn_prof_import_set_read(buf, 0)
    tot = max(1, buf[0])
    for i, name in NAMES.items():
        cyc = i in (0, 1, 3, 6, 8, 12, 13, 14, 16, 17, 18)
        print("%-34s %16d %s" % (name, buf[i], ("%5.1f%%" % (100.0 * buf[i] / tot)) if cyc else ""), flush=True)


if __name__ == "__main__":
    main()
