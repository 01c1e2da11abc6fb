"""Multi-GPU plumbing for the key-sharded flush window (one process per GPU).

Keys are partitioned the way veneur routes them to workers -- FNV-1a-32 digest of
(name, type, joined tags) modulo the number of consumers (server.go:655,
samplers/parser.go:213-304) -- so every rank aggregates a disjoint key set and the data
path needs no collective.  The only collectives are the bench's control plane: a barrier
around the timed region, the max of the per-rank elapsed times and the sum of samples.
They run over RCCL ("nccl") on GPUs and over gloo on CPU (the multi-process tests).
"""
import os

import numpy as np


def env_world():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_of(digest, n_shards):
    """Owner rank of each key: digest % n (veneur's worker routing applied to GPUs)."""
    return (np.asarray(digest, dtype=np.uint32) % np.uint32(n_shards)).astype(np.int64)


class Group:
    """torch.distributed process group wrapper; world_size 1 means no group at all."""

    def __init__(self, backend=None, local_rank=0):
        self.world, self.rank, _ = env_world()
        self.dist = None
        self.device = None
        if self.world <= 1:
            return
        import torch
        import torch.distributed as td
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            self.device = torch.device("cuda", local_rank)
            td.init_process_group("nccl", device_id=self.device)
        else:
            self.device = torch.device("cpu")
            td.init_process_group("gloo")
        self.dist = td

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x, op):
        if self.dist is None:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x):
        return self._reduce(x, self.dist.ReduceOp.MAX if self.dist else None)

    def sum(self, x):
        return self._reduce(x, self.dist.ReduceOp.SUM if self.dist else None)

    def broadcast_object(self, obj, src=0):
        """src's object on every rank (small control data only)."""
        if self.dist is None:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=src)
        return box[0]

    def gather_object(self, obj):
        """All ranks' objects on every rank (small control data only)."""
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def route_stream(d, rank, n_shards):
    """The records of a synthetic stream (engine.synth output) whose key this rank owns,
    in arrival order, keeping the stream's slot numbering: what veneur's per-worker
    channel would deliver to consumer `rank` of `n_shards`."""
    own = [shard_of(d["digest_of_slot"][c], n_shards) == rank for c in range(4)]
    out = dict(d)
    for c, (sk, cols) in enumerate((("c_slot", ("c_val", "c_rate")), ("g_slot", ("g_val",)),
                                    ("h_slot", ("h_val", "h_rate")))):
        m = own[c][d[sk]] if len(d[sk]) else np.zeros(0, bool)
        out[sk] = d[sk][m]
        for col in cols:
            out[col] = d[col][m]
    m = own[3][d["s_slot"]] if len(d["s_slot"]) else np.zeros(0, bool)
    off = d["s_off"].astype(np.int64)
    idx = np.nonzero(m)[0]
    lens = off[idx + 1] - off[idx]
    new_off = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(lens, out=new_off[1:])
    take = np.repeat(off[idx] - new_off[:-1], lens) + np.arange(new_off[-1])
    out["s_slot"] = d["s_slot"][m]
    out["s_off"] = new_off.astype(np.uint32)
    out["s_bytes"] = d["s_bytes"][take]
    return out


# ---------------------------------------------------------------- hot keys spanning GPUs
# One very hot key would pin one GPU under key routing, so its samples may instead be spread
# over every rank (each rank holds the key in the same slot).  At flush the partial states
# meet on the key's owner rank (digest % N), the way a global veneur combines what its locals
# forward (flusher.go:264-353 -> handlers_global.go:53-63 -> worker.go:230-268):
#   histograms / timers  every rank exports its partial digest (Histo.Export = GobEncode), one
#                        all-gather moves the payloads, the owner imports them
#                        (Histo.Combine = MergingDigest.Merge): the all-gather + re-merge
#   sets                 the same with MarshalBinary / Sketch.Merge: an exact union
#   counters             all-reduce(sum) of the int64 values
# On GPUs the payloads stay in HBM end to end: export writes device bytes, RCCL (backend
# "nccl" = RCCL over xGMI) all-gathers them, import reads them in place.  On CPU (gloo) the
# same protocol runs over host tensors for the multi-process tests.

def _allgather_payloads(group, payload, off):
    """All ranks' (bytes, offsets) of one export: payload is a 1-D uint8 tensor on the group's
    device, off its payload offsets (numpy int64, n+1; n may differ between ranks)."""
    import torch
    td = group.dist
    dev = group.device
    meta = torch.tensor([payload.numel(), len(off)], dtype=torch.int64, device=dev)
    metas = [torch.zeros_like(meta) for _ in range(group.world)]
    td.all_gather(metas, meta)
    sizes = [int(m[0].item()) for m in metas]
    noffs = [int(m[1].item()) for m in metas]
    mx = max(1, max(sizes))
    pad = torch.zeros(mx, dtype=torch.uint8, device=dev)
    pad[:payload.numel()] = payload
    bufs = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(group.world)]
    td.all_gather(bufs, pad)
    mo = max(noffs)
    offt = torch.zeros(mo, dtype=torch.int64, device=dev)
    offt[:len(off)] = torch.from_numpy(np.ascontiguousarray(off, dtype=np.int64)).to(dev)
    offs = [torch.empty_like(offt) for _ in range(group.world)]
    td.all_gather(offs, offt)
    return [(bufs[r][:sizes[r]], offs[r][:noffs[r]].cpu().numpy()) for r in range(group.world)]


def _select(buf, off, idx):
    """The payloads idx of (buf, off), concatenated: (bytes tensor, offsets)."""
    import torch
    lens = off[np.asarray(idx) + 1] - off[np.asarray(idx)]
    new_off = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(lens, out=new_off[1:])
    if len(idx) == 0 or new_off[-1] == 0:
        return torch.zeros(1, dtype=torch.uint8, device=buf.device), new_off
    return torch.cat([buf[int(off[i]):int(off[i + 1])] for i in idx]), new_off


def exchange_hot(group, store, cls, slots, owners):
    """Move every rank's partial state of the hot keys `slots` (class "histo" or "set") to the
    owner rank owners[i] and merge it there, other ranks in rank order.  A rank exports only
    the keys it does not own (export mutates: GobEncode merges pending temps, as in Go), so
    the owner's own partial is the first contribution.  store: an EngineStore (GPU) or any
    object with export(cls, slots) -> (uint8 tensor, offsets) and
    import_(cls, slots, bytes tensor, offsets)."""
    slots = np.ascontiguousarray(slots, dtype=np.uint32)
    owners = np.asarray(owners, dtype=np.int64)
    if group.dist is None or len(slots) == 0:
        return
    payload, off = store.export(cls, slots[owners != group.rank])
    gathered = _allgather_payloads(group, payload, off)
    if not np.any(owners == group.rank):
        return
    for r in range(group.world):
        if r == group.rank:
            continue
        sent = owners != r                         # what rank r exported, in slot order
        pick = np.nonzero(owners[sent] == group.rank)[0]
        if len(pick) == 0:
            continue
        buf, off_r = gathered[r]
        sel, sel_off = _select(buf, off_r, pick)
        store.import_(cls, slots[sent][pick], sel, sel_off)


def allreduce_counters(group, values):
    """Sum of every rank's int64 counter values of the hot counters (Counter.Combine)."""
    v = np.ascontiguousarray(values, dtype=np.int64)
    if group.dist is None:
        return v
    import torch
    t = torch.from_numpy(v.copy()).to(group.device)
    group.dist.all_reduce(t, op=group.dist.ReduceOp.SUM)
    return t.cpu().numpy()


class EngineStore:
    """exchange_hot's view of a GPU engine: device-resident export / import (no host copy)."""

    def __init__(self, engine):
        self.e = engine

    def export(self, cls, slots):
        import ctypes as C

        import torch

        from . import _abi as A
        fn = A.lib.vn_export_histos if cls == "histo" else A.lib.vn_export_sets
        s = np.ascontiguousarray(slots, dtype=np.uint32)
        x = A.Export()
        self.e._check(fn(self.e.h, s.ctypes.data_as(A.u32p), len(s), C.byref(x)))
        off = np.ctypeslib.as_array(x.off, shape=(x.n + 1,)).astype(np.int64)
        buf = torch.empty(max(1, int(off[-1])), dtype=torch.uint8, device="cuda:%d" % self.e.device)
        if off[-1]:
            rc = A.lib.vn_device_copy(self.e.device, C.c_void_p(buf.data_ptr()), C.c_void_p(x.dev_bytes), int(off[-1]))
            if rc != 0:
                raise RuntimeError("vn_device_copy failed")
        return buf[:int(off[-1])], off

    def import_(self, cls, slots, data, off):
        import ctypes as C

        import torch

        from . import _abi as A
        dev = data.device
        st = torch.from_numpy(np.ascontiguousarray(slots, dtype=np.uint32).view(np.int32)).to(dev)
        ot = torch.from_numpy(np.ascontiguousarray(off, dtype=np.int64)).to(dev)
        fn = A.lib.vn_import_histos_device if cls == "histo" else A.lib.vn_import_sets_device
        torch.cuda.synchronize(dev)
        self.e._check(fn(self.e.h, C.c_void_p(st.data_ptr()), C.c_void_p(ot.data_ptr()),
                         C.c_void_p(data.data_ptr()), len(slots)))
