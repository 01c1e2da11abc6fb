"""Host-side handle of the MI355X engine (one per GPU / worker group).

Mirrors the part of veneur's Worker the hot path owns: ProcessMetric batches go in with
`ingest`, ImportMetric values with `import_*`, and `flush` returns what Worker.Flush +
the samplers' Flush methods compute (worker.go:187-298, samplers/samplers.go:125-526).
"""
import ctypes as C
import warnings
from dataclasses import dataclass

import numpy as np

from . import _abi as A


class EngineError(RuntimeError):
    pass


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


@dataclass
class FlushOutput:
    counter_slot: np.ndarray
    counter_value: np.ndarray      # int64 Counter.value
    gauge_slot: np.ndarray
    gauge_value: np.ndarray
    histo_slot: np.ndarray
    histo_stats: np.ndarray        # [n, 8]: weight, min, max, sum, rsum, digest min/max/count
    histo_quantiles: np.ndarray    # [n, n_percentiles]
    set_slot: np.ndarray
    set_estimate: np.ndarray       # uint64 Sketch.Estimate()
    set_sparse: np.ndarray
    samples_processed: int
    samples_imported: int
    warn_flags: int = 0            # the caller's misuse this window (VN_WARN_*); the flush completed


def _arr(ptr, n, dt, shape=None):
    if n == 0:
        return np.zeros((0,) if shape is None else (0,) + shape, dt)
    a = np.ctypeslib.as_array(ptr, shape=(n * (int(np.prod(shape)) if shape else 1),)).copy()
    a = a.view(dt) if a.dtype != dt else a
    return a.reshape((n,) + shape) if shape else a


class Engine:
    def __init__(self, capacity, compression=100.0, percentiles=(0.5, 0.9, 0.99, 0.999), max_batch_records=1 << 20,
                 max_batch_member_bytes=0, device=0, exact_threshold=0, hot_prefix=0, piece_growth=0,
                 split_max_records=0, split_compression=0.0, replay_reserved_cus=0, max_class_records=None):
        """max_class_records: (counter, gauge, histo, set) record caps of one ingest call, each <=
        max_batch_records (0 or None: max_batch_records); they size each class's buffers."""
        cfg = A.Config()
        cfg.replay_reserved_cus = int(replay_reserved_cus)
        cfg.split_max_records = int(split_max_records)
        cfg.split_compression = float(split_compression)
        if exact_threshold and exact_threshold != 0xFFFFFFFF and not A.FAST_MODE:
            raise EngineError("exact_threshold=%d is the t-digest fast mode, which %s is built without "
                              "(a VARIANT_FLAGS=-DVN_FAST_MODE=1 build carries it)" % (exact_threshold, A.LIB_PATH))
        cfg.histo_exact_threshold = int(exact_threshold)
        cfg.histo_hot_prefix = int(hot_prefix)
        cfg.histo_piece_growth = int(piece_growth)
        cfg.device = device
        for i, c in enumerate(capacity):
            cfg.capacity[i] = int(c)
        cfg.compression = float(compression)
        cfg.n_percentiles = len(percentiles)
        for i, p in enumerate(percentiles):
            cfg.percentiles[i] = float(p)
        cfg.max_batch_records = int(max_batch_records)
        cfg.max_batch_member_bytes = int(max_batch_member_bytes)
        for i, c in enumerate(max_class_records or ()):
            cfg.max_batch_class_records[i] = int(c)
        self.percentiles = tuple(float(p) for p in percentiles)
        self.capacity = tuple(int(c) for c in capacity)
        self.device = device
        # the engine's effective limits (capi.hip vn_engine_create)
        self.max_batch_records = int(max_batch_records) or (1 << 20)
        self.max_class_records = tuple(int(c) or self.max_batch_records for c in (max_class_records or (0,) * 4))
        self.max_batch_member_bytes = max(int(max_batch_member_bytes) or self.max_batch_records * 16,
                                          self.max_batch_records * 8)
        h = C.c_void_p()
        rc = A.lib.vn_engine_create(C.byref(cfg), C.byref(h))
        self.h = h
        if rc != 0:
            msg = A.lib.vn_last_error(h).decode() if h else "vn_engine_create failed"
            if h:
                A.lib.vn_engine_destroy(h)
            self.h = None
            raise EngineError("%s (rc=%d)" % (msg, rc))

    def close(self):
        if getattr(self, "h", None):
            A.lib.vn_engine_destroy(self.h)
            self.h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc):
        if rc != 0:
            raise EngineError("%s (rc=%d)" % (A.lib.vn_last_error(self.h).decode(), rc))

    # ---------------------------------------------------------------- ingest
    def ingest(self, counters=None, gauges=None, histos=None, sets=None, set_hashes=None):
        """One ProcessMetric batch (host arrays, arrival order per class).

        counters=(slot, value, rate), gauges=(slot, value), histos=(slot, value, rate),
        sets=(slot, member_off[n+1], member_bytes) or set_hashes=(slot, hash64)."""
        b = A.Batch()
        keep = []
        if counters is not None:
            s, v, r = _c(counters[0], np.uint32), _c(counters[1], np.float64), _c(counters[2], np.float32)
            keep += [s, v, r]
            b.n_counter, b.counter_slot, b.counter_value, b.counter_rate = len(s), _p(s), _p(v), _p(r)
        if gauges is not None:
            s, v = _c(gauges[0], np.uint32), _c(gauges[1], np.float64)
            keep += [s, v]
            b.n_gauge, b.gauge_slot, b.gauge_value = len(s), _p(s), _p(v)
        if histos is not None:
            s, v, r = _c(histos[0], np.uint32), _c(histos[1], np.float64), _c(histos[2], np.float32)
            keep += [s, v, r]
            b.n_histo, b.histo_slot, b.histo_value, b.histo_rate = len(s), _p(s), _p(v), _p(r)
        if sets is not None:
            s, o, m = _c(sets[0], np.uint32), _c(sets[1], np.uint32), _c(sets[2], np.uint8)
            if m.size == 0:
                m = np.zeros(1, np.uint8)
            keep += [s, o, m]
            b.n_set, b.set_slot, b.set_member_off, b.set_member_bytes = len(s), _p(s), _p(o), _p(m)
        elif set_hashes is not None:
            s, hs = _c(set_hashes[0], np.uint32), _c(set_hashes[1], np.uint64)
            keep += [s, hs]
            b.n_set, b.set_slot, b.set_hash = len(s), _p(s), _p(hs)
        self._check(A.lib.vn_ingest_host(self.h, C.byref(b)))

    def stage(self):
        """vn_stage_acquire: numpy views of the engine-owned pinned staging buffers."""
        st = A.Stage()
        self._check(A.lib.vn_stage_acquire(self.h, C.byref(st)))
        n, nb = int(st.capacity), int(st.member_bytes_capacity)
        v = lambda p, k: np.ctypeslib.as_array(p, shape=(k,))
        return {"counter_slot": v(st.counter_slot, n), "counter_value": v(st.counter_value, n),
                "counter_rate": v(st.counter_rate, n), "gauge_slot": v(st.gauge_slot, n),
                "gauge_value": v(st.gauge_value, n), "histo_slot": v(st.histo_slot, n),
                "histo_value": v(st.histo_value, n), "histo_rate": v(st.histo_rate, n),
                "set_slot": v(st.set_slot, n), "set_member_off": v(st.set_member_off, n + 1),
                "set_member_bytes": v(st.set_member_bytes, nb)}

    def submit(self, n_counter=0, n_gauge=0, n_histo=0, n_set=0, n_set_member_bytes=0):
        """vn_submit: ingest the records the caller wrote into the pinned stage."""
        c = A.BatchCounts(n_counter, n_gauge, n_histo, n_set, n_set_member_bytes)
        self._check(A.lib.vn_submit(self.h, C.byref(c)))

    def ingest_device(self, batch):
        """Ingest a batch whose arrays are already resident in device memory (A.Batch)."""
        self._check(A.lib.vn_ingest(self.h, C.byref(batch)))

    # ------------------------------------------------------------ split (hot) keys
    def set_comm(self, comm):
        """Exchange split keys over comm (a Comm) at flush; None: a group of one."""
        self.comm = comm
        self._check(A.lib.vn_engine_set_comm(self.h, comm.h if comm is not None else None))

    def split_keys(self, cls, slots, owners):
        """The window's split keys of class cls (0 counter, 2 histo, 3 set): this rank's slots
        and owner ranks, in the group-wide order."""
        s, o = _c(slots, np.uint32), _c(owners, np.uint32)
        if len(s) != len(o):
            raise ValueError("one owner per split key")
        self._check(A.lib.vn_split_keys(self.h, int(cls), s.ctypes.data_as(A.u32p), o.ctypes.data_as(A.u32p), len(s)))

    def hot_detect(self, stride=1):
        """vn_hot_detect: count every stride-th ingested record per slot (0: off, 1: exact)."""
        self._check(A.lib.vn_hot_detect(self.h, int(stride)))

    def hot_keys(self, cls, min_count, cap=64):
        """vn_hot_keys after a flush: (slots, estimated counts) of class cls at or above
        min_count in the flushed window, hottest first, at most cap."""
        slots = np.zeros(max(1, cap), np.uint32)
        counts = np.zeros(max(1, cap), np.uint64)
        n = C.c_uint32(0)
        self._check(A.lib.vn_hot_keys(self.h, int(cls), int(min_count), int(cap), slots.ctypes.data_as(A.u32p),
                                      counts.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(n)))
        return slots[:n.value].copy(), counts[:n.value].copy()

    def split_close(self):
        """vn_split_close: this window's split records are all in; their combine starts now."""
        self._check(A.lib.vn_split_close(self.h))

    def split_combine(self):
        """vn_split_combine: meet the group now (collective); vn_flush does it otherwise."""
        self._check(A.lib.vn_split_combine(self.h))

    def ingest_split_device(self, batch):
        """vn_ingest_split of an A.SplitBatch whose arrays are in device memory."""
        self._check(A.lib.vn_ingest_split(self.h, C.byref(batch)))

    def ingest_split(self, histos=None, set_hashes=None, sets=None):
        """Split-key records from host arrays (copied to the device first): histos=(key, value,
        rate), set_hashes=(key, hash64) or sets=(key, member_off[n+1], member_bytes)."""
        bufs = []

        def dev(a):
            b = DeviceBuffer(a, device=self.device)
            bufs.append(b)
            return b.ptr.value

        b = A.SplitBatch()
        try:
            if histos is not None:
                k, v, r = _c(histos[0], np.uint32), _c(histos[1], np.float64), _c(histos[2], np.float32)
                b.n_histo = len(k)
                if len(k):
                    b.histo_key, b.histo_value, b.histo_rate = dev(k), dev(v), dev(r)
            if set_hashes is not None:
                k, hs = _c(set_hashes[0], np.uint32), _c(set_hashes[1], np.uint64)
                b.n_set = len(k)
                if len(k):
                    b.set_key, b.set_hash = dev(k), dev(hs)
            elif sets is not None:
                k, o, m = _c(sets[0], np.uint32), _c(sets[1], np.uint32), _c(sets[2], np.uint8)
                b.n_set = len(k)
                if len(k):
                    b.set_key, b.set_member_off, b.set_member_bytes = dev(k), dev(o), dev(m if m.size else
                                                                                    np.zeros(1, np.uint8))
            self.ingest_split_device(b)
            A.lib.vn_device_synchronize(self.device)
        finally:
            for x in bufs:
                x.free()

    def import_counters(self, slot, values):
        s, v = _c(slot, np.uint32), _c(values, np.int64)
        self._check(A.lib.vn_import_counters(self.h, s.ctypes.data_as(A.u32p), v.ctypes.data_as(A.i64p), len(s)))

    def import_gauges(self, slot, values):
        s, v = _c(slot, np.uint32), _c(values, np.float64)
        self._check(A.lib.vn_import_gauges(self.h, s.ctypes.data_as(A.u32p), v.ctypes.data_as(A.f64p), len(s)))

    @staticmethod
    def _payloads(slot, payloads):
        s = _c(slot, np.uint32)
        if len(s) != len(payloads):
            raise ValueError("one slot per payload")
        off = np.zeros(len(payloads) + 1, np.uint64)
        off[1:] = np.cumsum([len(p) for p in payloads])
        blob = np.frombuffer(b"".join(payloads) or b"\0", np.uint8).copy()
        return s, off, blob

    def import_histos(self, slot, payloads):
        """ImportMetric of histograms/timers: Histo.Combine of each GobEncode()d digest
        (samplers.go:519-526) into histo slot[i], in order."""
        s, off, blob = self._payloads(slot, payloads)
        self._check(A.lib.vn_import_histos(self.h, s.ctypes.data_as(A.u32p), off.ctypes.data_as(A.u64p),
                                           blob.ctypes.data_as(A.u8p), len(s)))

    def import_sets(self, slot, payloads):
        """ImportMetric of sets: Set.Combine of each MarshalBinary()d sketch
        (samplers.go:313-325) into set slot[i], in order."""
        s, off, blob = self._payloads(slot, payloads)
        self._check(A.lib.vn_import_sets(self.h, s.ctypes.data_as(A.u32p), off.ctypes.data_as(A.u64p),
                                         blob.ctypes.data_as(A.u8p), len(s)))

    def _query(self, kind, slot, arg):
        s, a = _c(np.atleast_1d(slot), np.uint32), _c(np.atleast_1d(arg), np.float64)
        s, a = np.broadcast_arrays(s, a)
        s, a = np.ascontiguousarray(s), np.ascontiguousarray(a)
        out = np.zeros(len(s))
        self._check(A.lib.vn_histo_query(self.h, kind, s.ctypes.data_as(A.u32p), a.ctypes.data_as(A.f64p), len(s),
                                         out.ctypes.data_as(A.f64p)))
        return out

    def quantile(self, slot, q):
        """MergingDigest.Quantile of histo slot(s) in the current window (merging_digest.go:283-313)."""
        return self._query(0, slot, q)

    def cdf(self, slot, x):
        """MergingDigest.CDF of histo slot(s) in the current window (merging_digest.go:247-279)."""
        return self._query(1, slot, x)

    def _export(self, fn, slot):
        s = _c(np.atleast_1d(slot), np.uint32)
        x = A.Export()
        self._check(fn(self.h, s.ctypes.data_as(A.u32p), len(s), C.byref(x)))
        if x.n == 0:
            return []
        off = np.ctypeslib.as_array(x.off, shape=(x.n + 1,)).copy()
        blob = np.ctypeslib.as_array(x.bytes, shape=(max(1, int(off[-1])),)).tobytes()
        return [blob[off[i]:off[i + 1]] for i in range(x.n)]

    def export_raw(self, cls, slot):
        """Export (cls 2 histo, 3 set) of slot[] as (offsets u64[n+1], bytes u8) host copies."""
        s = _c(np.atleast_1d(slot), np.uint32)
        x = A.Export()
        fn = A.lib.vn_export_histos if cls == 2 else A.lib.vn_export_sets
        self._check(fn(self.h, s.ctypes.data_as(A.u32p), len(s), C.byref(x)))
        off = np.ctypeslib.as_array(x.off, shape=(x.n + 1,)).copy()
        blob = np.ctypeslib.as_array(x.bytes, shape=(max(1, int(off[-1])),)).copy()
        return off, blob

    def export_device(self, cls, slot):
        """Export (cls 2 histo, 3 set) of slot[] into a DeviceBuffer of its own: (offsets u64[n+1]
        host copy, DeviceBuffer of the bytes, zero-copy numpy view of the engine's pinned host
        bytes -- valid until the engine's next export)."""
        s = _c(np.atleast_1d(slot), np.uint32)
        x = A.Export()
        fn = A.lib.vn_export_histos if cls == 2 else A.lib.vn_export_sets
        self._check(fn(self.h, s.ctypes.data_as(A.u32p), len(s), C.byref(x)))
        off = np.ctypeslib.as_array(x.off, shape=(x.n + 1,)).copy()
        nb = int(off[-1])
        buf = DeviceBuffer.empty(nb, self.device)
        if nb and A.lib.vn_device_copy(self.device, buf.ptr, C.c_void_p(x.dev_bytes),
                                       nb) != 0:
            raise EngineError("device copy of the export failed")
        view = np.ctypeslib.as_array(x.bytes, shape=(max(1, nb),))
        return off, buf, view

    def import_device(self, cls, slot_ptr, off_ptr, bytes_ptr, n):
        """vn_import_histos_device / vn_import_sets_device (cls 2 / 3) of device-resident payloads."""
        fn = A.lib.vn_import_histos_device if cls == 2 else A.lib.vn_import_sets_device
        self._check(fn(self.h, slot_ptr, off_ptr, bytes_ptr, int(n)))

    def export_histos(self, slot):
        """Histo.Export: GobEncode()d digest of each histo slot (merges its pending temps)."""
        return self._export(A.lib.vn_export_histos, slot)

    def export_sets(self, slot):
        """Set.Export: MarshalBinary()d sketch of each set slot."""
        return self._export(A.lib.vn_export_sets, slot)

    def sync(self):
        self._check(A.lib.vn_sync(self.h))

    # ---------------------------------------------------------------- flush
    def flush_raw(self, histo_quantile_mask=None, set_estimate_mask=None):
        out = A.FlushResult()
        if histo_quantile_mask is None and set_estimate_mask is None:
            self._check(A.lib.vn_flush(self.h, C.byref(out)))
            return out
        masks = []
        for m, cap in ((histo_quantile_mask, self.capacity[2]), (set_estimate_mask, self.capacity[3])):
            if m is None:
                masks.append(None)
            else:
                a = np.zeros(max(cap, 1), np.uint8)
                m = np.asarray(m, np.uint8)
                a[:len(m)] = m[:cap]
                masks.append(a)
        self._check(A.lib.vn_flush_masked(self.h, *(None if a is None else a.ctypes.data_as(A.u8p) for a in masks),
                                          C.byref(out)))
        return out

    def flush(self, histo_quantile_mask=None, set_estimate_mask=None) -> FlushOutput:
        """Worker.Flush + sampler flush math; the masks (per slot, 1 = compute) select which
        histograms get percentiles and which sets an estimate (a local veneur, vn_flush_masked)."""
        return flush_output(self.flush_raw(histo_quantile_mask, set_estimate_mask), len(self.percentiles))

    # ---------------------------------------------------------------- introspection
    def read_histo(self, slot, cap=4096):
        m = np.zeros(cap)
        w = np.zeros(cap)
        st = np.zeros(A.VN_HISTO_STATS)
        n = C.c_uint32()
        self._check(A.lib.vn_read_histo(self.h, slot, m.ctypes.data_as(A.f64p), w.ctypes.data_as(A.f64p), cap,
                                        C.byref(n), st.ctypes.data_as(A.f64p)))
        return m[:n.value], w[:n.value], st

    def read_set(self, slot):
        st = A.SetState()
        lc = np.zeros(16640, np.uint32)
        tc = np.zeros(256, np.uint32)
        regs = np.zeros(A.HLL_M, np.uint8)
        self._check(A.lib.vn_read_set(self.h, slot, C.byref(st), lc.ctypes.data_as(A.u32p), len(lc),
                                      tc.ctypes.data_as(A.u32p), len(tc), regs.ctypes.data_as(A.u8p)))
        d = {k: getattr(st, k) for k, _ in A.SetState._fields_ if k != "pad"}
        d["list"] = lc[:st.list_count].copy() if st.sparse else np.zeros(0, np.uint32)
        d["tmp"] = np.sort(tc[:st.tmp_count]) if st.sparse else np.zeros(0, np.uint32)
        d["registers"] = regs if not st.sparse else None
        return d

    # ---------------------------------------------------------------- timing
    def timing_enable(self, on=True):
        self._check(A.lib.vn_timing_enable(self.h, int(bool(on))))

    def timing(self):
        t = A.Timing()
        self._check(A.lib.vn_get_timing(self.h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in A.Timing._fields_}

    def import_counts(self, reset=False):
        """Import contributions decoded while timing was on (vn_import_counts): histo payloads,
        their centroids, set payloads, dense set payloads, sparse set codes."""
        out = (C.c_uint64 * 5)()
        self._check(A.lib.vn_import_counts(self.h, out, int(bool(reset))))
        return dict(zip(("histo_payloads", "centroids", "set_payloads", "dense_sets", "sparse_codes"),
                        (int(v) for v in out)))


def flush_output(o, npct) -> FlushOutput:
    """A vn_flush_result (engine-owned pinned arrays, valid until that engine's next flush) copied
    into a FlushOutput of numpy arrays."""
    out = FlushOutput(
        counter_slot=_arr(o.counter_slot, o.n_counter, np.uint32),
        counter_value=_arr(o.counter_value, o.n_counter, np.int64),
        gauge_slot=_arr(o.gauge_slot, o.n_gauge, np.uint32),
        gauge_value=_arr(o.gauge_value, o.n_gauge, np.float64),
        histo_slot=_arr(o.histo_slot, o.n_histo, np.uint32),
        histo_stats=_arr(o.histo_stats, o.n_histo, np.float64, (A.VN_HISTO_STATS,)),
        histo_quantiles=(_arr(o.histo_quantiles, o.n_histo, np.float64, (npct,)) if npct
                         else np.zeros((o.n_histo, 0))),
        set_slot=_arr(o.set_slot, o.n_set, np.uint32),
        set_estimate=_arr(o.set_estimate, o.n_set, np.uint64),
        set_sparse=_arr(o.set_sparse, o.n_set, np.uint8),
        samples_processed=o.samples_processed,
        samples_imported=o.samples_imported,
        warn_flags=int(o.warn_flags),
    )
    if out.warn_flags & A.VN_WARN_SPLIT_TOUCHED:
        warnings.warn("a split key's slot also received vn_ingest records or imports this window (its "
                      "records go through vn_ingest_split); the split combine's state was kept", RuntimeWarning)
    return out


class Comm:
    """A group of engines exchanging split keys: RCCL (one process per GPU) or in-process."""

    def __init__(self, h):
        self.h = h

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * A.VN_COMM_ID_BYTES)()
        if A.lib.vn_comm_unique_id(buf) != 0:
            raise EngineError("vn_comm_unique_id failed (librccl)")
        return bytes(buf)

    @classmethod
    def rccl(cls, uid, nranks, rank, device):
        buf = (C.c_uint8 * A.VN_COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        rc = A.lib.vn_comm_init(buf, nranks, rank, device, C.byref(h))
        if rc != 0:
            msg = A.lib.vn_comm_last_error(h).decode() if h else ""
            if h:
                A.lib.vn_comm_destroy(h)
            raise EngineError("vn_comm_init failed (rc=%d): %s" % (rc, msg))
        return cls(h)

    @classmethod
    def local(cls, nranks, device=0):
        hs = (C.c_void_p * nranks)()
        if A.lib.vn_comm_init_local(nranks, device, hs) != 0:
            raise EngineError("vn_comm_init_local failed")
        return [cls(C.c_void_p(h)) for h in hs]

    @property
    def rank(self):
        return A.lib.vn_comm_rank(self.h)

    @property
    def nranks(self):
        return A.lib.vn_comm_nranks(self.h)

    def allreduce_f64(self, values, op, device=0):
        """Control-plane all-reduce of a few doubles (through device memory)."""
        v = np.ascontiguousarray(values, np.float64)
        b = DeviceBuffer(v, device=device)
        try:
            if A.lib.vn_comm_allreduce(self.h, b.ptr, b.ptr, len(v), A.VN_DT_F64, op) != 0:
                raise EngineError("vn_comm_allreduce: %s" % A.lib.vn_comm_last_error(self.h).decode())
            out = np.zeros_like(v)
            A.lib.vn_device_synchronize(device)
            A.lib.vn_copy_to_host(device, out.ctypes.data_as(C.c_void_p), b.ptr, v.nbytes)
            return out
        finally:
            b.free()

    def close(self):
        if getattr(self, "h", None):
            A.lib.vn_comm_destroy(self.h)
            self.h = None


def metro64_device(members, seed=1337, device=0):
    """metro.Hash64 of every member on the GPU (kernel-level known-answer entry point)."""
    blob = b"".join(members)
    off = np.zeros(len(members) + 1, np.uint32)
    off[1:] = np.cumsum([len(m) for m in members])
    buf = np.frombuffer(blob if blob else b"\0", np.uint8).copy()
    out = np.zeros(len(members), np.uint64)
    rc = A.lib.vn_metro64(device, buf.ctypes.data_as(A.u8p), off.ctypes.data_as(A.u32p), len(members), seed,
                          out.ctypes.data_as(A.u64p))
    if rc != 0:
        raise EngineError("vn_metro64 failed (rc=%d)" % rc)
    return out


def device_count():
    n = C.c_int(0)
    return n.value if A.lib.vn_device_count(C.byref(n)) == 0 else 0


class DeviceBuffer:
    """Device allocation owned by Python (bench inputs resident in HBM)."""

    def __init__(self, host_array, device=0):
        a = np.ascontiguousarray(host_array)
        self.nbytes = a.nbytes
        self.ptr = C.c_void_p()
        if A.lib.vn_device_alloc(device, max(1, a.nbytes), C.byref(self.ptr)) != 0:
            raise EngineError("device allocation of %d bytes failed" % a.nbytes)
        if a.nbytes and A.lib.vn_copy_to_device(device, self.ptr, a.ctypes.data_as(C.c_void_p), a.nbytes) != 0:
            raise EngineError("host to device copy failed")

    @classmethod
    def empty(cls, nbytes, device=0):
        """An uninitialised device allocation of nbytes."""
        b = cls.__new__(cls)
        b.nbytes = int(nbytes)
        b.ptr = C.c_void_p()
        if A.lib.vn_device_alloc(device, max(1, b.nbytes), C.byref(b.ptr)) != 0:
            raise EngineError("device allocation of %d bytes failed" % b.nbytes)
        return b

    def free(self):
        if self.ptr:
            A.lib.vn_device_free(self.ptr)
            self.ptr = None

    __del__ = free


def synth(seed=1, n_keys=1000, zipf_s=1.0, mix=(0.4, 0.2, 0.25, 0.15), n_samples=100000, shard=0, n_shards=1,
          member_universe=50_000_000, rate_half=0.05, rate_tenth=0.05, histo_mu=3.912023005428146,
          histo_sigma=1.0, threads=0):
    """Synthetic DogStatsD-shaped stream (include/veneur_amd_synth.h) as numpy arrays."""
    cfg = A.SynthConfig(seed, n_keys, zipf_s, (C.c_double * 4)(*mix), n_samples, shard, n_shards, member_universe,
                        rate_half, rate_tenth, histo_mu, histo_sigma, threads)
    out = A.SynthOut()
    rc = A.lib.vn_synth_generate(C.byref(cfg), C.byref(out))
    if rc != 0:
        raise EngineError("vn_synth_generate failed (rc=%d)" % rc)
    try:
        n = [int(out.n[i]) for i in range(4)]
        cp = lambda p, k, dt: np.ctypeslib.as_array(p, shape=(k,)).astype(dt, copy=True) if k else np.zeros(0, dt)
        d = {
            "n_slots": tuple(int(out.n_slots[i]) for i in range(4)),
            "c_slot": cp(out.c_slot, n[0], np.uint32), "c_val": cp(out.c_val, n[0], np.float64),
            "c_rate": cp(out.c_rate, n[0], np.float32),
            "g_slot": cp(out.g_slot, n[1], np.uint32), "g_val": cp(out.g_val, n[1], np.float64),
            "h_slot": cp(out.h_slot, n[2], np.uint32), "h_val": cp(out.h_val, n[2], np.float64),
            "h_rate": cp(out.h_rate, n[2], np.float32),
            "s_slot": cp(out.s_slot, n[3], np.uint32), "s_off": cp(out.s_off, n[3] + 1, np.uint32),
            "s_bytes": cp(out.s_bytes, int(out.s_nbytes), np.uint8),
            "key_of_slot": [cp(out.key_of_slot[i], int(out.n_slots[i]), np.uint32) for i in range(4)],
            "digest_of_slot": [cp(out.digest_of_slot[i], int(out.n_slots[i]), np.uint32) for i in range(4)],
        }
    finally:
        A.lib.vn_synth_free(C.byref(out))
    return d


# ---------------------------------------------------------------- the C4 stream in HBM
C3_MIX = (0.4, 0.2, 0.25, 0.15)


def _dev_config(seed, n_keys, n_samples, rank, nranks, device, zipf_s=1.0, mix=C3_MIX, member_universe=50_000_000,
                rate_half=0.05, rate_tenth=0.05, histo_mu=3.912023005428146, histo_sigma=1.0, split=None):
    cfg = A.SynthDevConfig()
    cfg.seed, cfg.n_keys, cfg.zipf_s, cfg.n_samples = seed, n_keys, zipf_s, n_samples
    for i in range(4):
        cfg.mix[i] = mix[i]
    cfg.rank, cfg.nranks, cfg.member_universe = rank, nranks, member_universe
    cfg.rate_half, cfg.rate_tenth, cfg.histo_mu, cfg.histo_sigma = rate_half, rate_tenth, histo_mu, histo_sigma
    cfg.device = device
    keep = []
    for c in range(4):
        ks = np.ascontiguousarray((split or {}).get(c, np.zeros(0, np.uint32)), np.uint32)
        keep.append(ks)
        cfg.n_split[c] = len(ks)
        cfg.split_key[c] = ks.ctypes.data_as(A.u32p) if len(ks) else None
    return cfg, keep


def synth_key_counts(seed, n_keys, n_samples, n_positions, device=0, **kw):
    """Record count of every key over the first n_positions of the C4 stream (on the GPU)."""
    cfg, _ = _dev_config(seed, n_keys, n_samples, 0, 1, device, **kw)
    out = np.zeros(n_keys, np.uint32)
    if A.lib.vn_synth_key_counts(C.byref(cfg), n_positions, out.ctypes.data_as(A.u32p)) != 0:
        raise EngineError("vn_synth_key_counts failed")
    return out


class HostWindows:
    """vn_synth_hosts_device: the C5 local windows of hosts [host0, host0 + n_hosts) in HBM
    (slot (h - host0) * n_keys + k per class), as a device batch for one local engine."""

    def __init__(self, seed, host0, n_hosts, n_histo_keys, n_set_keys, device=0):
        cfg = A.SynthHostsConfig(seed, host0, n_hosts, n_histo_keys, n_set_keys, device)
        self.out = A.SynthHostsOut()
        rc = A.lib.vn_synth_hosts_device(C.byref(cfg), C.byref(self.out))
        if rc != 0:
            raise EngineError("vn_synth_hosts_device failed (rc=%d)" % rc)
        o = self.out
        self.batch = A.Batch()
        self.batch.n_histo, self.batch.histo_slot, self.batch.histo_value, self.batch.histo_rate = (
            o.n_histo, o.h_slot, o.h_val, o.h_rate)
        self.batch.n_set, self.batch.set_slot, self.batch.set_hash = o.n_set, o.s_slot, o.s_hash
        self.n_histo, self.n_set = int(o.n_histo), int(o.n_set)

    def free(self):
        if getattr(self, "out", None) is not None:
            A.lib.vn_synth_hosts_free(C.byref(self.out))
            self.out = None

    __del__ = free


class DeviceStream:
    """vn_synth_device: this rank's share of the C4 stream, resident in HBM."""

    def __init__(self, seed, n_keys, n_samples, rank, nranks, device=0, split=None, **kw):
        cfg, self._keep = _dev_config(seed, n_keys, n_samples, rank, nranks, device, split=split, **kw)
        self.out = A.SynthDevOut()
        self.device = device
        rc = A.lib.vn_synth_device(C.byref(cfg), C.byref(self.out))
        if rc != 0:
            raise EngineError("vn_synth_device failed (rc=%d)" % rc)
        o = self.out
        self.n_slots = tuple(int(o.n_slots[c]) for c in range(4))
        self.split_slot0 = tuple(int(o.split_slot0[c]) for c in range(4))
        self.n_split = tuple(int(cfg.n_split[c]) for c in range(4))
        cp = lambda p, k: np.ctypeslib.as_array(p, shape=(k,)).copy() if k else np.zeros(0, np.uint32)
        self.key_of_slot = [cp(o.key_of_slot[c], self.n_slots[c]) for c in range(4)]
        self.digest_of_slot = [cp(o.digest_of_slot[c], self.n_slots[c]) for c in range(4)]
        self.batch, self.split = o.batch, o.split
        self.counts = (int(o.batch.n_counter), int(o.batch.n_gauge), int(o.batch.n_histo), int(o.batch.n_set))
        self.split_counts = (int(o.split.n_histo), int(o.split.n_set))
        self.n_records = sum(self.counts) + sum(self.split_counts)
        self.counter_sum = int(o.counter_sum)
        self.histo_weight = float(o.histo_weight)

    def _host(self, ptr, n, dt):
        a = np.zeros(max(n, 0), dt)
        if n:
            A.lib.vn_copy_to_host(self.device, a.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), a.nbytes)
        return a

    def to_host(self):
        """The rank's records as host arrays, split records mapped to their local slots (one
        consumer's view of the same stream: per-key arrival order is kept)."""
        b, s = self.batch, self.split
        h = self._host
        d = {"c_slot": h(b.counter_slot, b.n_counter, np.uint32), "c_val": h(b.counter_value, b.n_counter, np.float64),
             "c_rate": h(b.counter_rate, b.n_counter, np.float32),
             "g_slot": h(b.gauge_slot, b.n_gauge, np.uint32), "g_val": h(b.gauge_value, b.n_gauge, np.float64)}
        hs = np.concatenate([h(b.histo_slot, b.n_histo, np.uint32),
                             h(s.histo_key, s.n_histo, np.uint32) + np.uint32(self.split_slot0[2])])
        d["h_slot"] = hs
        d["h_val"] = np.concatenate([h(b.histo_value, b.n_histo, np.float64), h(s.histo_value, s.n_histo, np.float64)])
        d["h_rate"] = np.concatenate([h(b.histo_rate, b.n_histo, np.float32), h(s.histo_rate, s.n_histo, np.float32)])
        d["s_slot"] = np.concatenate([h(b.set_slot, b.n_set, np.uint32),
                                      h(s.set_key, s.n_set, np.uint32) + np.uint32(self.split_slot0[3])])
        mb = np.concatenate([h(b.set_member_bytes, b.n_set * 11, np.uint8),
                             h(s.set_member_bytes, s.n_set * 11, np.uint8)])
        d["s_bytes"] = mb
        d["s_off"] = (np.arange(len(d["s_slot"]) + 1, dtype=np.uint64) * 11).astype(np.uint32)
        d["n_slots"] = self.n_slots
        return d

    def free(self):
        if getattr(self, "out", None) is not None:
            A.lib.vn_synth_device_free(C.byref(self.out))
            self.out = None

    __del__ = free
