"""CPU restatement of the split-key combine of veneur_amd/csrc/split.hip (test infrastructure).

Each rank holds its share of a hot key's records -- record j of the key's window on rank j % N --
and the ranks meet over a torch.distributed group (gloo on CPU) exactly as the engine's ranks
meet over RCCL:
  counters   all-reduce(sum)
  sets       the first J records gathered and replayed in order (oracle Sketch.insert_hash),
             J growing while a key is still sparse with records beyond it; then the dense
             insert's rebase epochs: all-reduce min of every zero register's first filler,
             all-reduce min of the first rebase candidate after T_full, all-reduce max of the
             registers below it, the rebase on every rank alike
  histos     the first P records gathered and Add()ed in window order, their pending temps
             merged, then per geometric piece one mergeAllTemps of every rank's micro-centroids
             (its share of the piece compressed alone at delta_hi, MergingDigest.add_batch)
The oracle (oracle/, the restated Go) is both the building block and the single-consumer
reference the tests compare against.
"""
import numpy as np
import torch

import oracle

P_HOT, GROWTH, DELTA_HI, J0 = 4096, 25, 500.0, 12288
INF = np.iinfo(np.int64).max


def _allreduce(group, arr, op):
    t = torch.from_numpy(np.ascontiguousarray(arr, np.int64).copy())
    group.dist.all_reduce(t, op=op)
    return t.numpy()


def counters(group, values):
    return _allreduce(group, values, group.dist.ReduceOp.SUM)


def pos_val(hashes, p=14):
    """getPosVal (axiomhq utils.go:46-51): register index (top p bits), rho = clz(x << p | 1 << (p-1)) + 1."""
    x = np.asarray(hashes, np.uint64)
    idx = (x >> np.uint64(64 - p)).astype(np.int64)
    w = (x << np.uint64(p)) | np.uint64(1 << (p - 1))
    lz = np.zeros(len(x), np.int64)
    for s in (32, 16, 8, 4, 2, 1):  # count leading zeros by halving
        m = (w >> np.uint64(64 - s)) == 0
        lz += np.where(m, s, 0)
        w = np.where(m, w << np.uint64(s), w)
    return idx, lz + 1


def sets(group, share, total):
    """share: this rank's hashes of one split set key in window order; total: the key's records
    over all ranks.  Returns (sparse, registers or None, b, sketch) of the combined state."""
    N, r = group.world, group.rank
    J = min(J0, max(total, 1))
    while True:
        m = -(-J // N)
        parts = group.gather_object(np.asarray(share[:m], np.uint64))
        sk = oracle.Sketch()
        for j in range(min(J, total)):
            sk.insert_hash(int(parts[j % N][j // N]))
        if not (sk.sparse and total > J):
            break
        J = min(J * 4, total)
    if total <= J:
        return sk
    idx, rho = pos_val(share)
    jj = r + N * np.arange(len(share), dtype=np.int64)
    regs = sk.registers().astype(np.int64)
    b = sk.b
    p0 = J
    while True:
        live = jj >= p0
        if (regs == 0).any():
            ff = np.full(len(regs), INF, np.int64)
            sel = live & (rho > b) & (regs[idx] == 0)
            np.minimum.at(ff, idx[sel], jj[sel])
            ff = _allreduce(group, ff, group.dist.ReduceOp.MIN)
            zf = ff[regs == 0]
            T = INF if (zf == INF).any() else int(zf.max())
        else:
            T = p0 - 1
        cand = INF
        if T != INF:
            c = live & (jj > T) & (((rho - b) & 0xFF) >= 16)
            cand = int(jj[c].min()) if c.any() else INF
        cand = int(_allreduce(group, [cand], group.dist.ReduceOp.MIN)[0])
        W = regs.copy()
        sel = live & (jj < cand) & (rho > b)
        np.maximum.at(W, idx[sel], np.minimum(rho[sel] - b, 15))
        regs = _allreduce(group, W, group.dist.ReduceOp.MAX)
        if cand == INF:
            break
        # the candidate record: its (index, rho) from the rank that holds it
        hold = np.nonzero(jj == cand)[0]
        pr = np.array([int(idx[hold[0]]), int(rho[hold[0]])] if len(hold) else [-1, -1], np.int64)
        pr = _allreduce(group, pr, group.dist.ReduceOp.MAX)
        db = int(regs.min())
        b += db
        regs -= db
        if pr[1] > b:
            regs[pr[0]] = max(regs[pr[0]], min(pr[1] - b, 15))
        p0 = cand + 1
    sk.sparse = False
    sk.b = b
    for i in np.nonzero(regs != sk.registers())[0]:
        sk.reg_set(int(i), int(regs[i]))
    return sk


def pieces(n, P=P_HOT, g=GROWTH):
    b = [P]
    while b[-1] < n:
        b.append(b[-1] + max(1, b[-1] * g // 100))
    return np.array(b, np.int64)


def histo(group, vals, wts, total, owner):
    """vals/wts: this rank's share of one split histogram in window order.  Returns the owner's
    combined MergingDigest (None elsewhere)."""
    N, r = group.world, group.rank
    jj = r + N * np.arange(len(vals), dtype=np.int64)
    pre = jj < P_HOT
    prefix = group.gather_object((jj[pre], vals[pre], wts[pre]))
    bounds = pieces(total)
    g = np.searchsorted(bounds, jj[~pre], side="right") - 1
    micro = []
    for piece in range(len(bounds) - 1):
        sel = g == piece
        if not sel.any():
            micro.append((np.zeros(0), np.zeros(0)))
            continue
        md = oracle.MergingDigest(DELTA_HI)
        md.add_batch(vals[~pre][sel], wts[~pre][sel])
        micro.append(md.centroids())
    allmicro = group.gather_object(micro)
    if r != owner:
        return None
    j = np.concatenate([p[0] for p in prefix])
    o = np.argsort(j, kind="stable")
    td = oracle.MergingDigest(100.0)
    td.add_many(np.concatenate([p[1] for p in prefix])[o], np.concatenate([p[2] for p in prefix])[o])
    td.quantile(0.5)  # Quantile's mergeAllTemps: the pending temps merged before the pieces
    for piece in range(len(bounds) - 1):
        m = np.concatenate([allmicro[q][piece][0] for q in range(N)])
        w = np.concatenate([allmicro[q][piece][1] for q in range(N)])
        if len(m):
            td.add_batch(m, w)
    return td
