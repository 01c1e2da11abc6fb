import sys, numpy as np
sys.path.insert(0, '/root/repo')
import oracle
from tools.tdigest_study import PCT, quantiles, rank_err, sample
from multiprocessing import Pool
def one(a):
    n, seed = a
    rng = np.random.default_rng(seed)
    v, w = sample(n, rng)
    go = oracle.MergingDigest(100.0); go.add_many(v, w); qg = quantiles(go)
    p = rng.permutation(n)
    g2 = oracle.MergingDigest(100.0); g2.add_many(v[p], w[p]); q2 = quantiles(g2)
    # same order, merge every 84 (two temp buffers at once)
    g3 = oracle.MergingDigest(100.0)
    for i in range(0, n, 84): g3.add_batch(v[i:i+84], w[i:i+84])
    q3 = quantiles(g3)
    # swap one adjacent pair of samples near the start
    v4, w4 = v.copy(), w.copy(); v4[[10, 11]] = v4[[11, 10]]; w4[[10, 11]] = w4[[11, 10]]
    g4 = oracle.MergingDigest(100.0); g4.add_many(v4, w4); q4 = quantiles(g4)
    return [rank_err(v, w, q2, qg), rank_err(v, w, q3, qg), rank_err(v, w, q4, qg)]
rng = np.random.default_rng(5)
sizes = np.exp(rng.uniform(np.log(32769), np.log(400000), 200)).astype(int)
with Pool(8) as pool:
    res = np.array(pool.map(one, [(int(n), 77 + i) for i, n in enumerate(sizes)]))
for i, name in enumerate(["permuted order", "merge every 84", "one adjacent swap"]):
    e = res[:, i]
    print("%-18s max %s frac>1e-3 %.3f mean %s" % (name, np.round(e.max(0), 5).tolist(), np.mean(e.max(1) > 1e-3), np.round(e.mean(0), 6).tolist()))
