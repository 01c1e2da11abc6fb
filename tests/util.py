"""Shared helpers for the parity tests: run the CPU oracle on a stream, compare results."""
import numpy as np
import pytest

import oracle


def _fast_mode_built():
    try:
        from veneur_amd import _abi
        return _abi.FAST_MODE
    except ImportError:
        return False


# the opt-in t-digest fast mode (exact_threshold > 0) is not in the shipped library
# (include/veneur_amd.h vn_build_flags): its tests run only against a VN_FAST_MODE=1 variant build
FAST_ONLY = pytest.mark.skipif(not _fast_mode_built(), reason="t-digest fast mode is a variant build (VN_FAST_MODE=1)")

PCT = (0.5, 0.9, 0.99, 0.999)


def run_oracle(stream, n_slots, batches=1, hashed=False):
    """Feed a stream dict (veneur_amd.synth layout) to the restated Go worker, in arrival
    order per class.  Returns the oracle Worker."""
    w = oracle.Worker(*n_slots)
    w.counter(stream["c_slot"], stream["c_val"], stream["c_rate"])
    w.gauge(stream["g_slot"], stream["g_val"])
    w.histo(stream["h_slot"], stream["h_val"], stream["h_rate"])
    if hashed:
        w.set_hashed(stream["s_slot"], stream["s_hash"])
    else:
        w.set(stream["s_slot"], stream["s_off"], stream["s_bytes"])
    return w


def split_batches(stream, nb):
    """Split each class stream into nb contiguous batches (arrival order preserved)."""
    out = []
    n = {k: len(stream[k]) for k in ("c_slot", "g_slot", "h_slot", "s_slot")}
    for b in range(nb):
        d = {}
        for cls, keys in (("c_slot", ("c_slot", "c_val", "c_rate")), ("g_slot", ("g_slot", "g_val")),
                          ("h_slot", ("h_slot", "h_val", "h_rate"))):
            lo, hi = n[cls] * b // nb, n[cls] * (b + 1) // nb
            for k in keys:
                d[k] = stream[k][lo:hi]
        lo, hi = n["s_slot"] * b // nb, n["s_slot"] * (b + 1) // nb
        d["s_slot"] = stream["s_slot"][lo:hi]
        if "s_hash" in stream:
            d["s_hash"] = stream["s_hash"][lo:hi]
        if "s_off" in stream:
            off = stream["s_off"][lo:hi + 1].astype(np.int64)
            d["s_bytes"] = stream["s_bytes"][off[0]:off[-1]]
            d["s_off"] = (off - off[0]).astype(np.uint32)
        out.append(d)
    return out


def engine_ingest(eng, d, hashed=False):
    kw = {}
    if len(d["c_slot"]):
        kw["counters"] = (d["c_slot"], d["c_val"], d["c_rate"])
    if len(d["g_slot"]):
        kw["gauges"] = (d["g_slot"], d["g_val"])
    if len(d["h_slot"]):
        kw["histos"] = (d["h_slot"], d["h_val"], d["h_rate"])
    if len(d["s_slot"]):
        if hashed:
            kw["set_hashes"] = (d["s_slot"], d["s_hash"])
        else:
            kw["sets"] = (d["s_slot"], d["s_off"], d["s_bytes"])
    eng.ingest(**kw)


def weighted_cdf(vals, wts):
    o = np.argsort(vals, kind="stable")
    v, w = vals[o], wts[o]
    cw = np.cumsum(w)
    tot = cw[-1]

    def F(x):
        i = np.searchsorted(v, x, side="right")
        return 0.0 if i == 0 else cw[i - 1] / tot
    return F


def rank_errors(stream, slots, eng_q, or_q, pct=PCT):
    """|F(q_engine) - F(q_oracle)| per (slot, percentile) with F the exact weighted CDF of
    the slot's samples (tdigest/analysis/main.go floatCDF, weighted by 1/rate)."""
    hs, hv, hr = stream["h_slot"], stream["h_val"], stream["h_rate"]
    order = np.argsort(hs, kind="stable")
    hs_o = hs[order]
    bounds = np.searchsorted(hs_o, slots, side="left"), np.searchsorted(hs_o, slots, side="right")
    errs = np.zeros((len(slots), len(pct)))
    for j, s in enumerate(slots):
        idx = order[bounds[0][j]:bounds[1][j]]
        F = weighted_cdf(hv[idx], (1.0 / hr[idx].astype(np.float32)).astype(np.float64))
        for k in range(len(pct)):
            errs[j, k] = abs(F(eng_q[j, k]) - F(or_q[j, k]))
    return errs
