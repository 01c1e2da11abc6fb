"""C3 at its configured size (BASELINE.json configs[2]): a mixed DogStatsD-shaped stream of 100M
samples over 1M keys (40 / 20 / 25 / 15 % counters / gauges / timers / sets by key, Zipf(1.0)
popularity, sample rates 1 / 0.5 / 0.1), one flush window on one GPU, against the restated Go
worker path (oracle, threaded by key digest as veneur's workers are) on the same records:

  * counters, gauges, set estimates: bit-exact for every key (worker.go:187-298,
    samplers.go:125-325, axiomhq hyperloglog);
  * histograms: LocalWeight / LocalMin / LocalMax and the digest's weight exact, LocalSum and
    LocalReciprocalSum within 1e-12 relative, every key's p50 / p90 / p99 / p99.9 bit-identical
    (samplers.go:346-498, merging_digest.go:97-313: every merge replayed exactly).
"""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

import veneur_amd as V  # noqa: E402  (fails loudly when the HIP library is missing)

PCT = (0.5, 0.9, 0.99, 0.999)
KEYS, SAMPLES, SEED = 1_000_000, 100_000_000, 3


def test_c3_full_size_bit_exact():
    s = V.DeviceStream(SEED, KEYS, SAMPLES, 0, 1, device=0, split=None)
    try:
        n_slots = tuple(max(1, x) for x in s.n_slots)
        with V.Engine(n_slots, compression=100.0, percentiles=PCT, max_batch_records=max(s.counts) + 1,
                      max_batch_member_bytes=s.counts[3] * 11 + 64) as e:
            e.ingest_device(s.batch)
            f = e.flush()
        d = s.to_host()
    finally:
        s.free()
    assert sum(s.counts) == SAMPLES
    streams = {k: d[k] for k in ("c_slot", "c_val", "c_rate", "g_slot", "g_val", "h_slot", "h_val", "h_rate",
                                 "s_slot", "s_off", "s_bytes")}
    threads = max(1, min(16, os.cpu_count() or 1))
    _, _, ref = oracle.baseline_run_full(threads, n_slots, streams, PCT)
    # counters / gauges / sets: every touched key, bit-exact
    assert np.array_equal(f.counter_slot, np.nonzero(ref["touched"][0])[0])
    assert np.array_equal(f.counter_value, ref["counter"][f.counter_slot])
    assert np.array_equal(f.gauge_slot, np.nonzero(ref["touched"][1])[0])
    assert np.array_equal(f.gauge_value, ref["gauge"][f.gauge_slot])
    assert np.array_equal(f.set_slot, np.nonzero(ref["touched"][3])[0])
    assert np.array_equal(f.set_estimate, ref["set_est"][f.set_slot])
    # histograms
    assert np.array_equal(f.histo_slot, np.nonzero(ref["touched"][2])[0])
    rs = ref["histo_stats"][f.histo_slot]
    assert np.array_equal(f.histo_stats[:, [0, 1, 2, 5, 6, 7]], rs[:, [0, 1, 2, 5, 6, 7]])
    with np.errstate(divide="ignore", invalid="ignore"):
        rel = np.abs(f.histo_stats[:, 3:5] - rs[:, 3:5]) / np.abs(rs[:, 3:5])
    assert np.nanmax(rel) <= 1e-12
    rq = ref["histo_q"][f.histo_slot]
    same = (f.histo_quantiles == rq) | (np.isnan(f.histo_quantiles) & np.isnan(rq))
    bad = np.nonzero(~np.all(same, axis=1))[0]
    assert len(bad) == 0, [(int(f.histo_slot[i]), f.histo_quantiles[i], rq[i]) for i in bad[:5]]
    assert len(f.histo_slot) > 100_000  # (the window touches most timer keys)
