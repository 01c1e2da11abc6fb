"""ctypes binding of the CPU oracle (oracle.c).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by veneur_amd.  See oracle.h for the
reference files each function restates.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(os.path.join(_HERE, "oracle.c")):
        build()
    return C.CDLL(_SO)


lib = _load()

u8p, u32p, u64p, i64p, f32p, f64p = (C.POINTER(t) for t in (C.c_uint8, C.c_uint32, C.c_uint64, C.c_int64, C.c_float, C.c_double))


def _sig(name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_sig("or_metro_hash64", C.c_uint64, C.c_char_p, C.c_size_t, C.c_uint64)
_sig("or_clz64", C.c_uint64, C.c_uint64)
_sig("or_fnv1a32", C.c_uint32, C.c_char_p, C.c_size_t, C.c_uint32)
_sig("or_go_log", C.c_double, C.c_double)
_sig("or_go_pow", C.c_double, C.c_double, C.c_double)
_sig("or_go_asin", C.c_double, C.c_double)
_sig("or_go_f64_to_i64", C.c_int64, C.c_double)
_sig("or_hll_new", C.c_void_p, C.c_uint8)
_sig("or_hll_free", None, C.c_void_p)
_sig("or_hll_clone", C.c_void_p, C.c_void_p)
_sig("or_hll_insert_hash", None, C.c_void_p, C.c_uint64)
_sig("or_hll_insert", None, C.c_void_p, C.c_char_p, C.c_size_t)
_sig("or_hll_estimate", C.c_uint64, C.c_void_p)
_sig("or_hll_merge", C.c_int, C.c_void_p, C.c_void_p)
_sig("or_hll_to_normal", None, C.c_void_p)
_sig("or_hll_merge_sparse", None, C.c_void_p)
_sig("or_hll_is_sparse", C.c_int, C.c_void_p)
_sig("or_hll_set_sparse_flag", None, C.c_void_p, C.c_int)
_sig("or_hll_p", C.c_uint8, C.c_void_p)
_sig("or_hll_b", C.c_uint8, C.c_void_p)
_sig("or_hll_set_b", None, C.c_void_p, C.c_uint8)
_sig("or_hll_nz", C.c_uint32, C.c_void_p)
_sig("or_hll_m", C.c_uint32, C.c_void_p)
_sig("or_hll_reg_get", C.c_uint8, C.c_void_p, C.c_uint32)
_sig("or_hll_reg_set", None, C.c_void_p, C.c_uint32, C.c_uint8)
_sig("or_hll_reg_rebase", None, C.c_void_p, C.c_uint8)
_sig("or_hll_list_codes", C.c_size_t, C.c_void_p, u32p, C.c_size_t)
_sig("or_hll_list_bytes", C.c_size_t, C.c_void_p)
_sig("or_hll_list_count", C.c_uint32, C.c_void_p)
_sig("or_hll_tmp_codes", C.c_size_t, C.c_void_p, u32p, C.c_size_t)
_sig("or_hll_tmp_len", C.c_size_t, C.c_void_p)
_sig("or_hll_tmp_add", None, C.c_void_p, C.c_uint32)
_sig("or_hll_list_append", None, C.c_void_p, C.c_uint32)
_sig("or_hll_tailcuts", C.c_size_t, C.c_void_p, u8p, C.c_size_t)
_sig("or_hll_marshal", C.c_size_t, C.c_void_p, u8p, C.c_size_t)
_sig("or_hll_unmarshal", C.c_int, C.c_void_p, C.c_char_p, C.c_size_t)
_sig("or_hll_encode_hash", C.c_uint32, C.c_uint64, C.c_uint8, C.c_uint8)
_sig("or_hll_decode_hash", None, C.c_uint32, C.c_uint8, C.c_uint8, u32p, u8p)
_sig("or_hll_get_pos_val", None, C.c_uint64, C.c_uint8, u64p, u8p)
_sig("or_td_new", C.c_void_p, C.c_double)
_sig("or_td_free", None, C.c_void_p)
_sig("or_td_add_batch", C.c_int, C.c_void_p, f64p, f64p, C.c_size_t)
_sig("or_td_add_many", C.c_long, C.c_void_p, f64p, f64p, C.c_size_t)
_sig("or_td_add", C.c_int, C.c_void_p, C.c_double, C.c_double)
_sig("or_td_quantile", C.c_double, C.c_void_p, C.c_double)
_sig("or_td_cdf", C.c_double, C.c_void_p, C.c_double)
_sig("or_td_min", C.c_double, C.c_void_p)
_sig("or_td_max", C.c_double, C.c_void_p)
_sig("or_td_count", C.c_double, C.c_void_p)
_sig("or_td_merge", None, C.c_void_p, C.c_void_p, i64p)
_sig("or_td_centroids", C.c_size_t, C.c_void_p, f64p, f64p, C.c_size_t)
_sig("or_td_main", C.c_size_t, C.c_void_p, f64p, f64p, C.c_size_t)
_sig("or_td_temp_len", C.c_size_t, C.c_void_p)
_sig("or_td_gob_encode", C.c_size_t, C.c_void_p, u8p, C.c_size_t)
_sig("or_td_gob_decode", C.c_int, C.c_void_p, C.c_char_p, C.c_size_t)
_sig("or_worker_new", C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32)
_sig("or_worker_free", None, C.c_void_p)
_sig("or_worker_counter", None, C.c_void_p, u32p, f64p, f32p, C.c_size_t)
_sig("or_worker_gauge", None, C.c_void_p, u32p, f64p, C.c_size_t)
_sig("or_worker_histo", None, C.c_void_p, u32p, f64p, f32p, C.c_size_t)
_sig("or_worker_set", None, C.c_void_p, u32p, u32p, u8p, C.c_size_t)
_sig("or_worker_set_hashed", None, C.c_void_p, u32p, u64p, C.c_size_t)
_sig("or_worker_import_counter", None, C.c_void_p, C.c_uint32, C.c_int64)
_sig("or_worker_import_gauge", None, C.c_void_p, C.c_uint32, C.c_double)
_sig("or_worker_import_set", C.c_int, C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t)
_sig("or_worker_import_histo", C.c_int, C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t, i64p)
_sig("or_worker_touched", C.c_int, C.c_void_p, C.c_int, C.c_uint32)
_sig("or_worker_counter_value", C.c_int64, C.c_void_p, C.c_uint32)
_sig("or_worker_gauge_value", C.c_double, C.c_void_p, C.c_uint32)
_sig("or_worker_histo_stats", None, C.c_void_p, C.c_uint32, f64p)
_sig("or_worker_histo_quantile", C.c_double, C.c_void_p, C.c_uint32, C.c_double)
_sig("or_worker_histo_centroids", C.c_size_t, C.c_void_p, C.c_uint32, f64p, f64p, C.c_size_t)
_sig("or_worker_set_estimate", C.c_uint64, C.c_void_p, C.c_uint32)
_sig("or_worker_histo_digest", C.c_void_p, C.c_void_p, C.c_uint32)
_sig("or_worker_set_sketch", C.c_void_p, C.c_void_p, C.c_uint32)
_sig("or_baseline_run", C.c_double, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
     u32p, f64p, f32p, C.c_size_t, u32p, f64p, C.c_size_t, u32p, f64p, f32p, C.c_size_t,
     u32p, u32p, u8p, C.c_size_t, f64p, C.c_int, f64p)


def ptr(a, t):
    """numpy array -> ctypes pointer (array must stay alive)."""
    return a.ctypes.data_as(t)


def metro64(b: bytes, seed: int = 1337) -> int:
    return lib.or_metro_hash64(b, len(b), seed)


def fnv1a32(*parts: bytes) -> int:
    h = 2166136261
    for p in parts:
        h = lib.or_fnv1a32(p, len(p), h)
    return h


def metric_digest(name: str, typ: str, joined_tags: str = "") -> int:
    """MetricKey digest: FNV-1a-32(name || type || joinedTags) (samplers/parser.go:213-304)."""
    return fnv1a32(name.encode(), typ.encode(), joined_tags.encode())


class Sketch:
    """axiomhq/hyperloglog.Sketch (oracle)."""

    def __init__(self, p=14, _h=None):
        self.h = _h if _h is not None else lib.or_hll_new(p)
        if not self.h:
            raise ValueError("p has to be >= 4 and <= 18")

    def __del__(self):
        if getattr(self, "h", None):
            lib.or_hll_free(self.h)
            self.h = None

    def clone(self):
        return Sketch(_h=lib.or_hll_clone(self.h))

    def insert(self, e: bytes):
        lib.or_hll_insert(self.h, e, len(e))

    def insert_hash(self, x: int):
        lib.or_hll_insert_hash(self.h, x)

    def estimate(self) -> int:
        return lib.or_hll_estimate(self.h)

    def merge(self, other):
        if lib.or_hll_merge(self.h, other.h if other is not None else None) != 0:
            raise ValueError("precisions must be equal")

    def to_normal(self):
        lib.or_hll_to_normal(self.h)

    def merge_sparse(self):
        lib.or_hll_merge_sparse(self.h)

    @property
    def sparse(self):
        return bool(lib.or_hll_is_sparse(self.h))

    @sparse.setter
    def sparse(self, v):
        lib.or_hll_set_sparse_flag(self.h, int(bool(v)))

    @property
    def p(self):
        return lib.or_hll_p(self.h)

    @property
    def b(self):
        return lib.or_hll_b(self.h)

    @b.setter
    def b(self, v):
        lib.or_hll_set_b(self.h, v)

    @property
    def nz(self):
        return lib.or_hll_nz(self.h)

    @property
    def m(self):
        return lib.or_hll_m(self.h)

    def reg_get(self, i):
        return lib.or_hll_reg_get(self.h, i)

    def reg_set(self, i, v):
        lib.or_hll_reg_set(self.h, i, v & 0xFF)

    def reg_rebase(self, d):
        lib.or_hll_reg_rebase(self.h, d)

    def registers(self) -> np.ndarray:
        """Unpacked registers (one byte per register)."""
        n = lib.or_hll_tailcuts(self.h, None, 0)
        tc = np.zeros(max(n, 1), np.uint8)
        lib.or_hll_tailcuts(self.h, ptr(tc, u8p), n)
        tc = tc[:n]
        out = np.empty(2 * n, np.uint8)
        out[0::2] = tc >> 4
        out[1::2] = tc & 15
        return out

    def list_codes(self) -> np.ndarray:
        n = lib.or_hll_list_codes(self.h, None, 0)
        a = np.zeros(max(n, 1), np.uint32)
        lib.or_hll_list_codes(self.h, ptr(a, u32p), n)
        return a[:n]

    def tmp_codes(self) -> np.ndarray:
        n = lib.or_hll_tmp_len(self.h)
        a = np.zeros(max(n, 1), np.uint32)
        lib.or_hll_tmp_codes(self.h, ptr(a, u32p), n)
        return a[:n]

    def list_bytes(self):
        return lib.or_hll_list_bytes(self.h)

    def list_count(self):
        return lib.or_hll_list_count(self.h)

    def tmp_add(self, code):
        lib.or_hll_tmp_add(self.h, code)

    def list_append(self, code):
        lib.or_hll_list_append(self.h, code)

    def marshal(self) -> bytes:
        n = lib.or_hll_marshal(self.h, None, 0)
        buf = np.zeros(n, np.uint8)
        lib.or_hll_marshal(self.h, ptr(buf, u8p), n)
        return buf.tobytes()

    def unmarshal(self, data: bytes):
        rc = lib.or_hll_unmarshal(self.h, data, len(data))
        if rc != 0:
            raise ValueError("bad sketch encoding (%d)" % rc)


def encode_hash(x, p, pp=25):
    return lib.or_hll_encode_hash(x, p, pp)


def decode_hash(k, p, pp=25):
    i = C.c_uint32()
    r = C.c_uint8()
    lib.or_hll_decode_hash(k, p, pp, C.byref(i), C.byref(r))
    return i.value, r.value


def get_pos_val(x, p):
    i = C.c_uint64()
    r = C.c_uint8()
    lib.or_hll_get_pos_val(x, p, C.byref(i), C.byref(r))
    return i.value, r.value


class MergingDigest:
    """tdigest.MergingDigest (oracle)."""

    def __init__(self, compression=100.0):
        self.td = lib.or_td_new(compression)

    def __del__(self):
        if getattr(self, "td", None):
            lib.or_td_free(self.td)
            self.td = None

    def add(self, v, w=1.0):
        if lib.or_td_add(self.td, v, w) != 0:
            raise ValueError("invalid value added")

    def add_many(self, values, weights):
        v = np.ascontiguousarray(values, np.float64)
        w = np.ascontiguousarray(weights, np.float64)
        if lib.or_td_add_many(self.td, ptr(v, f64p), ptr(w, f64p), len(v)) >= 0:
            raise ValueError("invalid value added")

    def add_batch(self, values, weights):
        """Study helper (not a reference function): one mergeAllTemps of all samples."""
        v = np.ascontiguousarray(values, np.float64)
        w = np.ascontiguousarray(weights, np.float64)
        if lib.or_td_add_batch(self.td, ptr(v, f64p), ptr(w, f64p), len(v)) != 0:
            raise MemoryError("or_td_add_batch")

    def quantile(self, q):
        if q < 0 or q > 1:
            raise ValueError("quantile out of bounds")
        return lib.or_td_quantile(self.td, q)

    def cdf(self, x):
        return lib.or_td_cdf(self.td, x)

    def min(self):
        return lib.or_td_min(self.td)

    def max(self):
        return lib.or_td_max(self.td)

    def count(self):
        return lib.or_td_count(self.td)

    def merge(self, other, perm=None):
        if perm is None:
            lib.or_td_merge(self.td, other.td, None)
        else:
            p = np.ascontiguousarray(perm, np.int64)
            lib.or_td_merge(self.td, other.td, ptr(p, i64p))

    def centroids(self):
        n = lib.or_td_centroids(self.td, None, None, 0)
        m = np.zeros(max(n, 1))
        w = np.zeros(max(n, 1))
        lib.or_td_centroids(self.td, ptr(m, f64p), ptr(w, f64p), n)
        return m[:n], w[:n]

    def main_centroids(self):
        """The main centroids without merging the pending temps (a replay's state between calls)."""
        n = lib.or_td_main(self.td, None, None, 0)
        m = np.zeros(max(n, 1))
        w = np.zeros(max(n, 1))
        lib.or_td_main(self.td, ptr(m, f64p), ptr(w, f64p), n)
        return m[:n], w[:n]

    def gob_encode(self) -> bytes:
        n = lib.or_td_gob_encode(self.td, None, 0)
        if n == 0:
            n = 1 << 20
        buf = np.zeros(n, np.uint8)
        k = lib.or_td_gob_encode(self.td, ptr(buf, u8p), n)
        return buf[:k].tobytes()

    def gob_decode(self, data: bytes):
        if lib.or_td_gob_decode(self.td, data, len(data)) != 0:
            raise ValueError("gob decode failed")


class Worker:
    """Restated Worker.ProcessMetric / ImportMetric over per-class slot tables (oracle)."""

    def __init__(self, n_counter, n_gauge, n_histo, n_set):
        self.w = lib.or_worker_new(n_counter, n_gauge, n_histo, n_set)
        self.n = (n_counter, n_gauge, n_histo, n_set)

    def __del__(self):
        if getattr(self, "w", None):
            lib.or_worker_free(self.w)
            self.w = None

    def counter(self, slot, value, rate):
        slot, value, rate = (np.ascontiguousarray(a, t) for a, t in ((slot, np.uint32), (value, np.float64), (rate, np.float32)))
        lib.or_worker_counter(self.w, ptr(slot, u32p), ptr(value, f64p), ptr(rate, f32p), len(slot))

    def gauge(self, slot, value):
        slot, value = np.ascontiguousarray(slot, np.uint32), np.ascontiguousarray(value, np.float64)
        lib.or_worker_gauge(self.w, ptr(slot, u32p), ptr(value, f64p), len(slot))

    def histo(self, slot, value, rate):
        slot, value, rate = (np.ascontiguousarray(a, t) for a, t in ((slot, np.uint32), (value, np.float64), (rate, np.float32)))
        lib.or_worker_histo(self.w, ptr(slot, u32p), ptr(value, f64p), ptr(rate, f32p), len(slot))

    def set(self, slot, member_off, member_bytes):
        slot = np.ascontiguousarray(slot, np.uint32)
        off = np.ascontiguousarray(member_off, np.uint32)
        mb = np.ascontiguousarray(member_bytes, np.uint8)
        if mb.size == 0:
            mb = np.zeros(1, np.uint8)
        lib.or_worker_set(self.w, ptr(slot, u32p), ptr(off, u32p), ptr(mb, u8p), len(slot))

    def set_hashed(self, slot, hashes):
        slot, hashes = np.ascontiguousarray(slot, np.uint32), np.ascontiguousarray(hashes, np.uint64)
        lib.or_worker_set_hashed(self.w, ptr(slot, u32p), ptr(hashes, u64p), len(slot))

    def import_counter(self, slot, v):
        lib.or_worker_import_counter(self.w, slot, v)

    def import_gauge(self, slot, v):
        lib.or_worker_import_gauge(self.w, slot, v)

    def import_set(self, slot, data: bytes):
        return lib.or_worker_import_set(self.w, slot, data, len(data))

    def import_histo(self, slot, data: bytes, perm=None):
        if perm is None:
            return lib.or_worker_import_histo(self.w, slot, data, len(data), None)
        p = np.ascontiguousarray(perm, np.int64)
        return lib.or_worker_import_histo(self.w, slot, data, len(data), ptr(p, i64p))

    def touched(self, cls, slot):
        return bool(lib.or_worker_touched(self.w, cls, slot))

    def touched_slots(self, cls):
        return np.array([s for s in range(self.n[cls]) if lib.or_worker_touched(self.w, cls, s)], np.uint32)

    def counter_value(self, slot):
        return lib.or_worker_counter_value(self.w, slot)

    def gauge_value(self, slot):
        return lib.or_worker_gauge_value(self.w, slot)

    def histo_stats(self, slot):
        o = np.zeros(8)
        lib.or_worker_histo_stats(self.w, slot, ptr(o, f64p))
        return o

    def histo_quantile(self, slot, q):
        return lib.or_worker_histo_quantile(self.w, slot, q)

    def histo_cdf(self, slot, x):
        """MergingDigest.CDF of the slot's digest (merges its pending temps, as Go does)."""
        return lib.or_td_cdf(lib.or_worker_histo_digest(self.w, slot), x)

    def histo_centroids(self, slot):
        n = lib.or_worker_histo_centroids(self.w, slot, None, None, 0)
        m = np.zeros(max(n, 1))
        w = np.zeros(max(n, 1))
        lib.or_worker_histo_centroids(self.w, slot, ptr(m, f64p), ptr(w, f64p), n)
        return m[:n], w[:n]

    def set_estimate(self, slot):
        return lib.or_worker_set_estimate(self.w, slot)

    def histo_gob(self, slot) -> bytes:
        """Histo.Export of the slot: GobEncode of its digest (merges its pending temps)."""
        td = lib.or_worker_histo_digest(self.w, slot)
        buf = np.zeros(1 << 20, np.uint8)
        k = lib.or_td_gob_encode(td, ptr(buf, u8p), len(buf))
        return buf[:k].tobytes()

    def set_sketch(self, slot):
        """Borrowed view of the slot's sketch (do not outlive the worker)."""
        h = lib.or_worker_set_sketch(self.w, slot)
        if not h:
            return None
        sk = Sketch.__new__(Sketch)
        sk.h = lib.or_hll_clone(h)
        return sk


def baseline_run(nthreads, nslots, streams, percentiles):
    """Time the restated Go worker path (ProcessMetric for every record, then the flush).

    streams: dict with c_slot/c_val/c_rate, g_slot/g_val, h_slot/h_val/h_rate, s_slot/s_off/s_bytes.
    Returns (seconds, checksum)."""
    s = streams
    arr = {}
    for k, t in (("c_slot", np.uint32), ("c_val", np.float64), ("c_rate", np.float32), ("g_slot", np.uint32),
                 ("g_val", np.float64), ("h_slot", np.uint32), ("h_val", np.float64), ("h_rate", np.float32),
                 ("s_slot", np.uint32), ("s_off", np.uint32), ("s_bytes", np.uint8)):
        a = np.ascontiguousarray(s[k], t)
        if a.size == 0:
            a = np.zeros(1, t)
        arr[k] = a
    pct = np.ascontiguousarray(percentiles, np.float64)
    cs = np.zeros(1)
    secs = lib.or_baseline_run(
        nthreads, *nslots,
        ptr(arr["c_slot"], u32p), ptr(arr["c_val"], f64p), ptr(arr["c_rate"], f32p), len(s["c_slot"]),
        ptr(arr["g_slot"], u32p), ptr(arr["g_val"], f64p), len(s["g_slot"]),
        ptr(arr["h_slot"], u32p), ptr(arr["h_val"], f64p), ptr(arr["h_rate"], f32p), len(s["h_slot"]),
        ptr(arr["s_slot"], u32p), ptr(arr["s_off"], u32p), ptr(arr["s_bytes"], u8p), len(s["s_slot"]),
        ptr(pct, f64p), len(pct), ptr(cs, f64p))
    return secs, float(cs[0])


class BaselineOut(C.Structure):
    _fields_ = [("counter", i64p), ("gauge", f64p), ("histo_q", f64p), ("histo_stats", f64p), ("set_est", u64p),
                ("touched", u8p * 4)]


_sig("or_baseline_set_output", None, C.POINTER(BaselineOut))


def baseline_run_full(nthreads, nslots, streams, percentiles):
    """baseline_run that also returns every flushed value per slot (for full-scale parity)."""
    nc, ng, nh, ns = (max(1, int(x)) for x in nslots)
    out = {"counter": np.zeros(nc, np.int64), "gauge": np.zeros(ng), "histo_q": np.zeros((nh, len(percentiles))),
           "histo_stats": np.zeros((nh, 8)), "set_est": np.zeros(ns, np.uint64),
           "touched": [np.zeros(n, np.uint8) for n in (nc, ng, nh, ns)]}
    bo = BaselineOut(ptr(out["counter"], i64p), ptr(out["gauge"], f64p), ptr(out["histo_q"], f64p),
                     ptr(out["histo_stats"], f64p), ptr(out["set_est"], u64p),
                     (u8p * 4)(*[ptr(t, u8p) for t in out["touched"]]))
    lib.or_baseline_set_output(C.byref(bo))
    try:
        secs, cs = baseline_run(nthreads, nslots, streams, percentiles)
    finally:
        lib.or_baseline_set_output(None)
    return secs, cs, out
