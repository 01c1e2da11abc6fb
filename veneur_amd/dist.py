"""Multi-GPU plumbing for the key-sharded flush window (one process per GPU).

Keys are partitioned the way veneur routes them to workers -- FNV-1a-32 digest of
(name, type, joined tags) modulo the number of consumers (server.go:655,
samplers/parser.go:213-304) -- so every rank aggregates a disjoint key set and ordinary keys
need no collective.  Hot keys are split over the ranks and combined by the engines over RCCL
(make_comm, deal, hot_keys below; the exchange itself is in libveneur_amd.so).  The host control
plane -- barrier around the timed region, max of the per-rank times, the RCCL id -- is a
torch.distributed group, gloo on the host.
"""
import os
import threading

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
# A key too hot for one GPU is split: its records are dealt round-robin over the ranks by the
# key's window arrival index, and at flush the engines combine the partial states on the key's
# owner over RCCL (include/veneur_amd.h "multi-GPU", csrc/split.hip).  The data path lives in
# libveneur_amd.so; this module only supplies the host-side pieces around it.

def deal(n_records, n_ranks):
    """Rank of each of a split key's n_records window records: its arrival index j, j % N."""
    return np.arange(n_records, dtype=np.int64) % int(n_ranks)


def route_imports(metrics, rank, world):
    """This rank's share of imported JSONMetrics in arrival order: newJSONMetricsByWorker's worker
    index, digest % N of name, type and joined tags (http.go:71-139, worker.go MetricKey), with
    the GPUs as the workers.  Each key lands on exactly one rank, so a global veneur over N GPUs
    merges every import where the key lives, with no data-path collective."""
    from .worker import metric_digest
    return [m for m in metrics if metric_digest(m.key) % int(world) == int(rank)]


def pack_metrics(metrics):
    """JSONMetrics as one byte string (the chunk a rank is sent): per metric the five fields of
    samplers.JSONMetric, each length-prefixed -- name, type, tagstring, the tags, value."""
    import struct
    out = [struct.pack("<I", len(metrics))]
    for m in metrics:
        f = [m.key.name.encode("utf-8", "surrogatepass"), m.key.type.encode("utf-8", "surrogatepass"),
             m.key.joined_tags.encode("utf-8", "surrogatepass")]
        tags = [t.encode("utf-8", "surrogatepass") for t in m.tags]
        val = bytes(m.value) if m.value is not None else b""
        out.append(struct.pack("<IIIII", len(f[0]), len(f[1]), len(f[2]), len(tags), len(val)))
        out += f
        out += [struct.pack("<I", len(t)) + t for t in tags]
        out.append(val)
    return b"".join(out)


def unpack_metrics(buf):
    """pack_metrics' inverse: the JSONMetrics in their order."""
    import struct
    from .worker import JSONMetric, MetricKey
    mv = memoryview(buf)
    n, = struct.unpack_from("<I", mv, 0)
    p = 4
    out = []
    for _ in range(n):
        ln, lt, lj, nt, lv = struct.unpack_from("<IIIII", mv, p)
        p += 20
        name = bytes(mv[p:p + ln]).decode("utf-8", "surrogatepass")
        p += ln
        typ = bytes(mv[p:p + lt]).decode("utf-8", "surrogatepass")
        p += lt
        joined = bytes(mv[p:p + lj]).decode("utf-8", "surrogatepass")
        p += lj
        tags = []
        for _ in range(nt):
            l, = struct.unpack_from("<I", mv, p)
            tags.append(bytes(mv[p + 4:p + 4 + l]).decode("utf-8", "surrogatepass"))
            p += 4 + l
        out.append(JSONMetric(MetricKey(name, typ, joined), tags, bytes(mv[p:p + lv])))
        p += lv
    return out


class ImportRouter:
    """/import for a global veneur spread over the ranks of `group` (one process per GPU).

    The reference decodes a body once and hands each worker its chunk (handleImport ->
    unmarshalMetricsFromHTTP -> ImportMetrics -> newJSONMetricsByWorker, handlers_global.go:53-63,
    http.go:52-139).  Here the GPUs are the workers: the rank holding the HTTP listener (src)
    decodes every body once -- zlib and JSON on its host -- routes the JSONMetrics by digest % N
    (route_imports: the sort newJSONMetricsByWorker does, arrival order kept within a rank), and
    sends each rank its chunk over the host control plane.  Every rank then imports only the keys
    it owns, so no imported key spans ranks and the payload merge on the GPUs needs no collective.

    route(body, content_encoding) is called by every rank for every body (src passes the body,
    the others None); it returns (HTTP status, this rank's JSONMetrics).  decoded counts the
    bodies this rank decoded."""

    def __init__(self, group, src=0):
        self.group, self.src, self.decoded = group, int(src), 0

    def route(self, body=None, content_encoding=""):
        from .http_import import ImportRequestError, StatusAccepted, unmarshal_metrics_from_http
        g = self.group
        world, rank = max(1, g.world), g.rank if g.dist is not None else 0
        chunks, status = None, StatusAccepted
        if rank == self.src:
            self.decoded += 1
            try:
                ms = unmarshal_metrics_from_http(body, content_encoding)
            except ImportRequestError as e:
                import logging
                logging.getLogger("veneur_amd.http_import").error("Could not decode /import request (%s): %s",
                                                                  e.cause or "empty", e)
                ms, status = [], e.status
            chunks = [route_imports(ms, r, world) for r in range(world)]
        if g.dist is None:
            return status, chunks[0]
        import torch
        td = g.dist
        # the status and every chunk's size first, then each rank's chunk (gloo point to point)
        hdr = torch.zeros(world + 1, dtype=torch.int64)
        packed = None
        if rank == self.src:
            packed = [pack_metrics(c) for c in chunks]
            hdr[0] = status
            hdr[1:] = torch.tensor([len(b) for b in packed], dtype=torch.int64)
        td.broadcast(hdr, src=self.src)
        status = int(hdr[0])
        if rank == self.src:
            for r in range(world):
                if r != self.src:
                    td.send(torch.frombuffer(bytearray(packed[r]), dtype=torch.uint8), dst=r)
            return status, chunks[rank]
        buf = torch.empty(int(hdr[1 + rank]), dtype=torch.uint8)
        td.recv(buf, src=self.src)
        return status, unpack_metrics(buf.numpy().tobytes())


def hot_keys(counts, classes, thresholds, max_split=64):
    """Top keys by window count above their class threshold: {class: sorted key ids}.
    counts: records per key (e.g. the previous window's), classes: class of every key,
    thresholds: {class: count} for the classes that may split (counter 0, histo 2, set 3)."""
    counts = np.asarray(counts, np.float64)
    out = {}
    for c, thr in thresholds.items():
        ks = np.nonzero((classes == c) & (counts > thr))[0]
        ks = ks[np.argsort(-counts[ks], kind="stable")][:max_split]
        out[c] = np.sort(ks).astype(np.uint32)
    return out


def make_comm(group, device):
    """The engines' RCCL group: rank 0 draws the unique id, the host control plane (gloo)
    broadcasts it, every rank joins (vn_comm_init).  None for a group of one."""
    from .engine import Comm
    if group.dist is None:
        return None
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")  # one node: the bootstrap stays on loopback
    uid = Comm.unique_id() if group.rank == 0 else None
    uid = group.broadcast_object(uid)
    return Comm.rccl(uid, group.world, group.rank, device)


class InTurn:
    """Flush windows over D engines per rank: window i runs on engine i % D, each engine's windows
    in order in a host thread of its own (D > 1), as veneur's flush goroutine works on the swapped
    maps while the workers take the next interval (server.go Flush / worker.go Flush).  work(k, i,
    turn) calls `with turn(i):` around the part of window i that issues collectives (the split
    combine, one communicator per engine), so every rank enters them in window order: engine k's
    communicator sees windows k, k + D, ... on every rank, and no two communicators' collectives
    are ever issued in different orders on two ranks.  run(n) returns the n results in window
    order; a failure in any window ends the others' waits.

    turn(i, section) keeps one such order per section: `with turn(i, 1):` around window i's
    ingest staggers the engines (window i + 1's ingest starts once window i's has been issued),
    so their long replays, which start at the end of an ingest, do not all run at once."""

    def __init__(self, D, sections=2):
        self.D = D
        self.cv = threading.Condition()
        self.next = [0] * sections
        self.failed = False

    def turn(self, i, section=0):
        pipe = self

        class _T:
            def __enter__(self):
                with pipe.cv:
                    pipe.cv.wait_for(lambda: pipe.next[section] == i or pipe.failed)
                    if pipe.failed:
                        raise RuntimeError("an earlier window failed")

            def __exit__(self, *exc):
                with pipe.cv:
                    if exc[0] is None:
                        pipe.next[section] = i + 1
                    else:
                        pipe.failed = True  # (the other engines' waits end)
                    pipe.cv.notify_all()
                return False

        return _T()

    def run(self, n, work):
        self.next, self.failed = [0] * len(self.next), False
        out, errs = [None] * n, []
        if self.D == 1:
            for i in range(n):
                out[i] = work(0, i, self.turn)
            return out

        def worker(k):
            try:
                for i in range(k, n, self.D):
                    out[i] = work(k, i, self.turn)
            except BaseException as ex:
                errs.append(ex)
                with self.cv:
                    self.failed = True
                    self.cv.notify_all()

        th = [threading.Thread(target=worker, args=(k,)) for k in range(self.D)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errs:
            raise errs[0]
        return out
