"""The batched exact replay of long keys (histo_exact.hip merge_batch) against the restated Go
digest, compared as whole digests: the GobEncode of every key (merging_digest.go:361-380, pending
temps merged first) byte for byte, plus the quantiles.

Keys of >= 524288 samples in one ingest call take the batched kernel (kBatchMinLen); every key
below carries at least that many per call.  The distributions aim at its
special paths:
  * lognormal with C4's rate mix -- the steady state (flips restart a batch);
  * a falling trend -- a new minimum in most chunks: Z temps before main 0 that start the first
    centroid, main 0 joining it (merging_digest.go:216);
  * a rising trend -- temps past the last main;
  * integer values 0..999 and 7 distinct values -- ties between temps and means (a temp equal to
    a mean goes before it: merging_digest.go:169); the 7-value key never batches;
  * weights up to 1000 (rate 0.001) and values around zero.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

import veneur_amd as V  # noqa: E402  (fails loudly when the HIP library is missing)

PCT = (0.5, 0.9, 0.99, 0.999)


def _key(kind, n, rng):
    if kind == "lognormal":
        v = rng.lognormal(np.log(50.0), 1.0, n)
        r = np.asarray((1.0, 0.5, 0.1), np.float32)[rng.choice(3, n, p=(0.9, 0.05, 0.05))]
    elif kind == "falling":
        v = 1e6 - np.arange(n) * 3.0 + rng.normal(0, 50.0, n)
        r = np.ones(n, np.float32)
    elif kind == "rising":
        v = np.arange(n) * 0.5 + rng.exponential(20.0, n)
        r = np.ones(n, np.float32)
    elif kind == "ints":
        v = rng.integers(0, 1000, n).astype(np.float64)
        r = np.asarray((1.0, 0.5), np.float32)[rng.choice(2, n, p=(0.8, 0.2))]
    elif kind == "seven":
        v = rng.integers(0, 7, n).astype(np.float64)
        r = np.ones(n, np.float32)
    elif kind == "past2_30":
        # integer weights of 2^20 (rate 2^-20) carry the digest's total past 2^30 within a few
        # thousand samples; a few samples at rate 0.3 (weight float32(1/0.3), a 2^-23 multiple)
        # make some main weights non-integer: sums of such weights are exact only up to 2^30, so
        # the fast merges and batches must step aside there (MergeState::fint)
        v = rng.lognormal(np.log(50.0), 1.0, n)
        c = rng.choice(3, n, p=(0.6, 0.399, 0.001))
        r = np.asarray((1.0, 2.0 ** -20, 0.3), np.float32)[c]
    elif kind == "heavy":
        v = rng.normal(0.0, 1.0, n)
        r = np.asarray((1.0, 0.01, 0.001), np.float32)[rng.choice(3, n, p=(0.98, 0.01, 0.01))]
    else:
        raise ValueError(kind)
    return v, r


def _stream(kinds, n, seed, noise_keys=50, noise=20_000):
    rng = np.random.default_rng(seed)
    # the keys interleaved at random, each key's own samples in its generated order
    out_s = np.repeat(np.arange(len(kinds), dtype=np.uint32), n)
    rng.shuffle(out_s)
    out_v, out_r = np.empty(len(out_s)), np.empty(len(out_s), np.float32)
    for k, kind in enumerate(kinds):
        v, r = _key(kind, n, rng)
        at = out_s == k
        out_v[at] = v
        out_r[at] = r
    # then a tail of small keys
    ns = rng.integers(len(kinds), len(kinds) + noise_keys, noise).astype(np.uint32)
    nv = rng.lognormal(3.0, 1.0, noise)
    nr = np.ones(noise, np.float32)
    return (np.concatenate([out_s, ns]), np.concatenate([out_v, nv]), np.concatenate([out_r, nr]),
            len(kinds) + noise_keys)


def _check(kinds, n, seed, batches):
    slot, val, rate, nk = _stream(kinds, n, seed)
    w = oracle.Worker(1, 1, nk, 1)
    w.histo(slot, val, rate)
    with V.Engine((1, 1, nk, 1), percentiles=PCT, max_batch_records=len(slot) + 1) as e:
        cuts = np.linspace(0, len(slot), batches + 1).astype(int)
        for a, b in zip(cuts[:-1], cuts[1:]):
            e.ingest(histos=(slot[a:b], val[a:b], rate[a:b]))
        gobs = e.export_histos(np.arange(len(kinds), dtype=np.uint32))
        f = e.flush()
    for k, kind in enumerate(kinds):
        exp = w.histo_gob(k)
        if gobs[k] != exp:
            a, b = oracle.MergingDigest(100.0), oracle.MergingDigest(100.0)
            a.gob_decode(gobs[k])
            b.gob_decode(exp)
            (ma, wa), (mb, wb) = a.centroids(), b.centroids()
            n = min(len(ma), len(mb))
            bad = np.nonzero((ma[:n] != mb[:n]) | (wa[:n] != wb[:n]))[0]
            i = int(bad[0]) if len(bad) else n
            raise AssertionError("%s (key %d): %d centroids, expected %d; first difference at %d: %r vs %r"
                                 % (kind, k, len(ma), len(mb), i, (ma[i:i + 3], wa[i:i + 3]),
                                    (mb[i:i + 3], wb[i:i + 3])))
    got = {int(s): q for s, q in zip(f.histo_slot, f.histo_quantiles)}
    for k in range(nk):
        exp = np.array([w.histo_quantile(k, p) for p in PCT])
        assert np.array_equal(got[k], exp), (k, got[k], exp)


@pytest.mark.parametrize("batches", [1, 3])
def test_batched_replay_whole_digest_bit_exact(batches):
    _check(["lognormal", "falling", "rising", "ints", "seven", "heavy"], 600_000 * batches, 11 + batches, batches)


def test_weights_past_2_30_with_non_integer_weights_bit_exact():
    """a digest holding non-integer (2^-23-grid) weights whose total passes 2^30 --
    the fast paths' exact-sum bound for such weights -- stays the reference's digest, bit for bit
    (the batched and four-wave replays step aside past the bound)."""
    _check(["past2_30", "past2_30"], 600_000, 7, 1)  # (batched)
    _check(["past2_30"], 200_000, 8, 2)  # (four-wave: 100k per call)


def test_batched_replay_one_long_key_bit_exact():
    """one 2M-sample C4 key: ~47k merges, most of them in batches of up to 64"""
    _check(["lognormal"], 2_000_000, 5, 1)


def test_four_wave_replay_new_last_centroid_bit_exact():
    """Keys of 65536-524287 samples per call take the four-wave replay (merge_fast).  A rising
    stream piles its temps past the last main centroid until they must start one of their own: the
    predicted chain ("every temp joins the centroid before it") has to be checked against the last
    element even when no later start exists (a bug found by the whole-digest comparison in round 4)."""
    _check(["rising", "rising", "falling", "lognormal"], 81_362, 1, 1)
    _check(["rising"] * 3, 150_000, 2, 2)


@pytest.mark.parametrize("calls", [2, 3])
def test_replay_state_after_every_call_bit_exact(calls):
    """Round 6: a long key continuing in a later ingest call starts by merging its pending temps
    with the call's first samples.  After every call each key's main centroids (vn_read_histo,
    pending temps not merged) equal the restated Go digest fed the same prefix of its samples --
    the out-of-line four-wave merge that this first merge used to take halved the centroids of
    continuing keys (tools/probe/repro_batch3_calls.py)."""
    kinds = ["lognormal", "falling", "rising", "ints", "seven", "heavy"]
    slot, val, rate, nk = _stream(kinds, 600_000 * calls, 11 + calls)
    wts = (np.float32(1.0) / rate).astype(np.float64)
    cuts = np.linspace(0, len(slot), calls + 1).astype(int)
    with V.Engine((1, 1, nk, 1), percentiles=PCT, max_batch_records=len(slot) + 1) as e:
        for a, b in zip(cuts[:-1], cuts[1:]):
            e.ingest(histos=(slot[a:b], val[a:b], rate[a:b]))
            for k, kind in enumerate(kinds):
                sel = slot[:b] == k
                td = oracle.MergingDigest(100.0)
                td.add_many(val[:b][sel], wts[:b][sel])
                om, ow = td.main_centroids()
                gm, gw, st = e.read_histo(k)
                assert np.array_equal(gm, om) and np.array_equal(gw, ow), (kind, b, len(gm), len(om))
                assert st[7] == float(np.sum(ow))
