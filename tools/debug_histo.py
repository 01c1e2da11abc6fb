import sys, numpy as np
sys.path.insert(0, '.')
import veneur_amd as V, oracle
from tests.util import PCT, run_oracle, rank_errors, engine_ingest
d = V.synth(seed=21, n_keys=400, zipf_s=1.0, mix=(0, 0, 1, 0), n_samples=200_000)
n = d['n_slots']; w = run_oracle(d, n)
e = V.Engine(tuple(max(1,x) for x in n), percentiles=PCT, max_batch_records=1<<18)
engine_ingest(e, d)
cents = {}
for s in range(n[2]):
    cents[s] = e.read_histo(s)
f = e.flush()
oq = np.array([[w.histo_quantile(int(s), p) for p in PCT] for s in f.histo_slot])
errs = rank_errors(d, f.histo_slot, f.histo_quantiles, oq)
cnt = np.bincount(d['h_slot'], minlength=n[2])
worst = np.argsort(errs.max(axis=1))[::-1][:8]
for j in worst:
    s = int(f.histo_slot[j])
    m, wt, st = cents[s]; om, ow = w.histo_centroids(s)
    print('slot', s, 'n', cnt[s], 'err', errs[j], 'eng q', f.histo_quantiles[j], 'ref q', oq[j])
    print('   ncent eng', len(m), 'ref', len(om), 'W eng', wt.sum(), 'ref', ow.sum(), 'T', st[7])
    if len(m) < 12: print('   eng', m, wt, '\n   ref', om, ow)
small = cnt[f.histo_slot] <= 42
print('small keys max abs q diff', np.abs(f.histo_quantiles[small]-oq[small]).max())
print('err by pct max', errs.max(axis=0), 'mean', errs.mean(axis=0))
