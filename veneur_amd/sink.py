"""Flush egress for the Datadog sink, native (vn_datadog_flush, csrc/sink.cpp).

Server.Flush's metric output (flusher.go:168-230 generateInterMetrics, samplers.go:136-498 the
samplers' Flush) through the Datadog sink (sinks/datadog/datadog.go:77-106,160-213: routing,
counters as rates, sink tags, host:/device: tags, chunks of at most flushMaxPerBody) to the request
bodies PostHelper encodes (http/http.go:116-135), built in C++ straight from the engine's flush
result and the window's keys -- no InterMetric objects per key.  Worker.flush_datadog is the
operator API; tests/dd_restated.py restates the same chain in Python as the checker.
"""
import ctypes as C
import threading
import time

import numpy as np

from . import _abi as A

MAP_IDS = ("counters", "global_counters", "gauges", "global_gauges", "histograms", "local_histograms", "timers",
           "local_timers", "sets", "local_sets")


class SinkError(RuntimeError):
    pass


def keys_from_maps(maps):
    """The window's keys (map name -> {MetricKey: (slot, tags)}) as vn_keys arrays: per key its map
    id, slot, tag count, and name + joined tags in one arena (creation order within each map)."""
    from .worker import go_bytes
    mp, slot, nt, noff, nlen, tlen, blob = [], [], [], [], [], [], bytearray()
    for mid, name in enumerate(MAP_IDS):
        for key, (s, tags) in maps.get(name, {}).items():
            nb, tb = go_bytes(key.name), go_bytes(",".join(tags))
            mp.append(mid), slot.append(s), nt.append(len(tags)), noff.append(len(blob))
            nlen.append(len(nb)), tlen.append(len(tb))
            blob += nb + tb
    arrs = (np.array(mp, np.uint8), np.array(slot, np.uint32), np.array(nt, np.uint32), np.array(noff, np.uint64),
            np.array(nlen, np.uint32), np.array(tlen, np.uint32), np.frombuffer(bytes(blob) or b"\0", np.uint8))
    k = A.Keys(len(mp), *(a.ctypes.data_as(t) for a, t in zip(arrs, (A.u8p, A.u32p, A.u32p, A.u64p, A.u32p, A.u32p,
                                                                       A.u8p))))
    return k, arrs  # keep arrs alive with k


class DatadogSink:
    """vn_sink: owns the bodies of its last flush.  One sink may serve several flush threads (a
    Worker with D > 1 engines flushes each engine on its own thread): the vn_sink's body buffers
    are rewritten by every vn_datadog_flush, so a lock is held from the call until its bodies are
    copied out."""

    def __init__(self, interval=10.0, hostname="", tags=(), flush_max_per_body=5000):
        self.interval, self.hostname, self.tags = float(interval), hostname, list(tags)
        self.flush_max_per_body = int(flush_max_per_body)
        self.h = C.c_void_p()
        self._lock = threading.Lock()
        if A.lib.vn_sink_create(C.byref(self.h)) != 0:
            raise SinkError("vn_sink_create failed")

    def close(self):
        if self.h:
            A.lib.vn_sink_destroy(self.h)
            self.h = C.c_void_p()

    def bodies(self, flush_result, maps, engine_percentiles, histogram_percentiles, aggregates, is_local,
               timestamp=None):
        """[(ok, body bytes)] per chunk, plus (n_intermetrics, n_metrics)."""
        keys, keep = keys_from_maps(maps)
        cfg = A.DDConfig()
        cfg.interval = self.interval
        cfg.timestamp = int(time.time()) if timestamp is None else int(timestamp)
        cfg.is_local = 1 if is_local else 0
        cfg.aggregates = int(aggregates.value)
        hp = list(histogram_percentiles)
        cfg.n_percentiles = len(hp)
        for i, p in enumerate(hp):
            cfg.percentiles[i] = p
        ep = np.array(list(engine_percentiles) or [0.0], np.float64)
        cfg.engine_percentiles = ep.ctypes.data_as(A.f64p)
        hn = self.hostname.encode("utf-8", "surrogateescape")
        st = ",".join(self.tags).encode("utf-8", "surrogateescape")
        cfg.hostname, cfg.sink_tags, cfg.n_sink_tags = hn, st, len(self.tags)
        cfg.flush_max_per_body = self.flush_max_per_body
        out = A.DDPayload()
        with self._lock:  # (ctypes releases the GIL inside the call)
            rc = A.lib.vn_datadog_flush(self.h, C.byref(flush_result), C.byref(keys), C.byref(cfg), C.byref(out))
            if rc != 0:
                raise SinkError("vn_datadog_flush: %s" % A.lib.vn_sink_last_error(self.h).decode(errors="replace"))
            off = np.ctypeslib.as_array(out.body_off, shape=(out.n_bodies + 1,)).copy()
            status = np.ctypeslib.as_array(out.body_status, shape=(out.n_bodies,)).copy()
            raw = C.string_at(out.bytes, int(off[-1])) if off[-1] else b""
        del keep
        return ([(status[i] == 0, raw[off[i]:off[i + 1]]) for i in range(out.n_bodies)],
                (int(out.n_intermetrics), int(out.n_metrics)))
