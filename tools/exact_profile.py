#!/usr/bin/env python3
"""Per-phase cycle profile of the exact t-digest replay (GPU box; profiling build).

Runs one hot key (and optionally many cold keys alongside it) through the engine built
with -DVN_EXACT_PROF (make -C veneur_amd prof) and prints the clock64 cycles block 0 spent
per merge phase.  Usage: VN_LIB=libveneur_amd_prof.so python tools/exact_profile.py
"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("VN_LIB", "libveneur_amd_prof.so")
import veneur_amd as V  # noqa: E402
import veneur_amd._abi as A  # noqa: E402

A.lib.vn_prof_exact_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
NAMES = ["tempW", "rank+pos", "prefix+kin", "chain", "welford", "merges", "elements", "centroids", "kernel"]


def run(n_hot, n_cold_keys, cold_per_key, seed=1):
    rng = np.random.default_rng(seed)
    nk = 1 + n_cold_keys
    slots = np.concatenate([np.zeros(n_hot, np.uint32),
                            np.repeat(np.arange(1, nk, dtype=np.uint32), cold_per_key)])
    rng.shuffle(slots[n_hot:])
    vals = np.exp(rng.normal(3.9, 1.0, len(slots)))
    rates = np.ones(len(slots), np.float32)
    with V.Engine((1, 1, nk, 1), compression=100.0, percentiles=(0.5, 0.99),
                  max_batch_records=len(slots) + 1) as e:
        e.timing_enable(True)
        buf = (C.c_ulonglong * 64)()
        A.lib.vn_prof_exact_read(buf, 1)
        t0 = time.perf_counter()
        e.ingest(histos=(slots, vals, rates))
        e.sync()
        wall = time.perf_counter() - t0
        A.lib.vn_prof_exact_read(buf, 1)
        e.flush()
        t = e.timing()
    p = list(buf)
    merges = max(1, p[5])
    out = {"n_hot": n_hot, "cold_keys": n_cold_keys, "ms_ingest_histo": round(t["ms_ingest_histo"], 3), "wall_ms": round(wall * 1e3, 3),
           "merges": p[5], "avg_elements": round(p[6] / merges, 1), "avg_centroids": round(p[7] / merges, 1),
           "kernel_cycles_block0": p[8]}
    for i in range(5):
        out["cyc_per_merge_" + NAMES[i]] = round(p[i] / merges, 1)
    out["cyc_per_merge_total"] = round(sum(p[:5]) / merges, 1)
    for i, nme in zip(range(9, 12), ("chain.forced", "chain.predict+verify", "chain.walks")):
        out["cyc_" + nme] = round(p[i] / merges, 1)
    out["merges_walked"] = p[12]
    nb = max(1, p[23])
    out["batches"] = p[23]
    out["batch_committed"] = p[24]
    out["batch_avg_committed"] = round(p[24] / nb, 2)
    out["batch_avg_usable"] = round(p[26] / nb, 2)
    out["batch_avg_flagged"] = round(p[25] / nb, 2)
    out["batch_structural_rejects"] = p[22]
    # merge_batch phases (histo_exact.hip): totals, A pos search, B n table + offsets,
    # C1+E+C2 lists / Welford / bounds, F decisions + bound tests, G flagged tests, H commit
    for i, nme in zip((16, 17, 18, 19, 15, 20, 21, 48, 13), ("totals", "A_pos", "B_ntable", "C_offsets_K_bounds",
                                                            "D_lists", "E_welford_C2", "F_decisions", "G_flagged",
                                                            "H_commit")):
        out["batch_cyc_" + nme] = round(p[i] / nb, 1)
    out["batch_cyc_column0_welford"] = round(p[14] / nb, 1)
    out["batch_cyc_call"] = round(p[27] / nb, 1)
    for base, nme in ((36, "E"), (40, "C_rows"), (44, "C2_queue")):
        out["batch_cyc_" + nme + "_per_wave"] = [round(p[base + w] / nb, 1) for w in range(4)]
    out["batch_E_longest_list_per_wave"] = [round(p[56 + w] / nb, 1) for w in range(3)]
    out["study_columns"] = p[52]
    out["study_cheap_certified"] = p[53]
    out["study_exact_certified"] = p[54]
    out["batch_repair_rounds"] = p[32]
    out["batch_avg_repairs"] = round(p[32] / nb, 2)
    out["batch_cyc_repair"] = round(p[33] / nb, 1)
    out["batch_redone_columns"] = p[35]
    nr = max(1, p[32])
    out["repair_round_cyc"] = {"R1_flags": round(p[49] / nr, 1), "R1_slots_counts": round(p[34] / nr, 1), "R2_welford_c2": round(p[50] / nr, 1),
                               "R3_recheck": round(p[51] / nr, 1), "R4_first": round(p[55] / nr, 1),
                               "R2_per_wave": [round(p[60 + w] / nr, 1) for w in range(4)],
                               "chunks_after_flip": round(p[59] / nr, 1)}
    out["singles_after_reject"] = p[29]
    out["singles_after_reject_cyc"] = p[28]
    out["singles_unbatchable"] = p[31]
    out["singles_unbatchable_cyc"] = p[30]
    print(out, flush=True)


if __name__ == "__main__":
    # one hot key: with the default (exact) engine it replays on the four-wave kernel, whose
    # phases are A = merge-path positions + weight prefix, B = k values, C = forced starts and
    # walks, D = masks + Welford (merge_fast); the one-wave kernel reports the old phase names.
    # "short:N:K": block 0 is one of K + 1 keys of N samples each (N < 8192: the one-wave
    # replay, merge_sorted_fast: rank+pos, prefix+kin, chain, welford), the other K beside it
    for n in (sys.argv[1:] or ["1000000"]):
        if n.startswith("short:"):
            _, ns, nk = n.split(":")
            run(int(ns), int(nk), int(ns))
        else:
            run(int(n), 0, 0)
