"""indexEstimate on the GPU as the replays evaluate it (gomath.h index_estimate<true>: its
divisions without v_div_scale / v_div_fixup) against the full correctly rounded division
sequence (index_estimate<false>), bit for bit, over the q values a merge can produce: P / T of
exact prefixes (integers up to 2^40, 2^-23 multiples up to 2^30), uniform q, and the edges
(0, 1, 1/2 and their neighbours).  merging_digest.go:240-243."""
import ctypes as C

import numpy as np
import pytest

import veneur_amd._abi as A

pytestmark = pytest.mark.gpu


def _mismatches(q, delta=100.0):
    q = np.ascontiguousarray(q, np.float64)
    out = C.c_uint64(0)
    vals = np.zeros(2 * len(q))
    rc = A.lib.vn_diag_index_estimate(0, delta, q.ctypes.data_as(C.POINTER(C.c_double)), len(q), C.byref(out),
                                      vals.ctypes.data_as(C.POINTER(C.c_double)))
    assert rc == 0
    bad = np.nonzero(vals[0::2].view(np.uint64) != vals[1::2].view(np.uint64))[0]
    assert len(bad) == out.value
    if len(bad):
        print("mismatches:", out.value, [(float(q[i]).hex(), vals[2 * i], vals[2 * i + 1]) for i in bad[:20]])
    return out.value


def test_index_estimate_divisions_bit_identical():
    rng = np.random.default_rng(11)
    qs = [rng.random(2_000_000)]
    for top in (2 ** 16, 2 ** 30, 2 ** 40):  # P / T with integer prefixes
        T = rng.integers(1, top, 1_000_000, dtype=np.int64)
        P = (rng.random(len(T)) * (T + 1)).astype(np.int64).clip(0, T)
        qs.append(P.astype(np.float64) / T.astype(np.float64))
    T = rng.integers(1, 2 ** 53, 500_000, dtype=np.int64) * 2.0 ** -23  # 2^-23 multiples (float32 rates)
    P = np.floor(rng.random(len(T)) * T * 2 ** 23) * 2.0 ** -23
    qs.append(np.minimum(P / T, 1.0))
    k = np.arange(1, 4096, dtype=np.float64)
    eps = 2.0 ** -53
    qs.append(np.concatenate([[0.0, 1.0, 0.5], 0.5 + k * eps, 0.5 - k * eps, 1 - k * eps, k * eps, k * 2.0 ** -40,
                              1 - k * 2.0 ** -40, np.nextafter(0.5, [0.0, 1.0])]))
    q = np.concatenate(qs)
    assert ((q >= 0) & (q <= 1)).all()
    for delta in (100.0, 50.0, 1000.0):
        assert _mismatches(q, delta) == 0


def test_index_estimate_device_equals_go_restatement():
    """The device's indexEstimate (the replays' form) against Go's expression evaluated on the host
    -- compression * (math.Asin(2*q - 1)/math.Pi + 0.5) with the oracle's math.Asin restatement --
    bit for bit, over q = P / T of large totals (T past 2^30 and 2^31, P stepping by small
    weights: consecutive k values an ulp apart, where a difference would flip a chain decision)."""
    import math

    import oracle
    rng = np.random.default_rng(12)
    qs = [rng.random(200_000)]
    for T in (2344619302.3333325, 2.0 ** 31 + 0.5, 1.5 * 2.0 ** 30, 8.4e10, 123456.0):
        P = np.floor(rng.random(100_000) * T)
        P[:2000] = np.arange(2000) + np.floor(T * 0.3)
        qs.append(P / T)
    q = np.concatenate(qs)
    vals = np.zeros(2 * len(q))
    out = C.c_uint64(0)
    assert A.lib.vn_diag_index_estimate(0, 100.0, q.ctypes.data_as(C.POINTER(C.c_double)), len(q), C.byref(out),
                                        vals.ctypes.data_as(C.POINTER(C.c_double))) == 0
    dev = vals[1::2]
    host = np.array([100.0 * (oracle.lib.or_go_asin(2.0 * x - 1.0) / math.pi + 0.5) for x in q])
    bad = np.nonzero(dev.view(np.uint64) != host.view(np.uint64))[0]
    assert len(bad) == 0, (len(bad), [(float(q[i]).hex(), dev[i], host[i]) for i in bad[:8]])
