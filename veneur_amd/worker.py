"""veneur's Worker and samplers API over the HIP engine (host side of the drop-in boundary).

This mirrors the reference's operator interface for the aggregation path -- the same names,
argument meaning and error behaviour -- so that code written against veneur's Worker reads the
same here:

  worker.go:22-138   Worker, WorkerMetrics (10 maps by type x scope), Upsert
  worker.go:187-227  Worker.ProcessMetric(UDPMetric)
  worker.go:230-268  Worker.ImportMetric(JSONMetric)
  worker.go:271-298  Worker.Flush() -> WorkerMetrics (swap, processed/imported reset)
  samplers/samplers.go:45-122   InterMetric, MetricType, Aggregate, HistogramAggregates, routeInfo
  samplers/samplers.go:136-526  Counter/Gauge/Set/Histo .Flush and .Export
  samplers/parser.go:21-43      UDPMetric, MetricKey, MetricScope
  parser.go:213-304, server.go:655, http.go:52-139   Digest routing and ImportMetrics chunking

What differs is where the work happens: ProcessMetric interns the MetricKey to a class-local
slot of the window (the map lookup of Upsert) and appends (slot, value, rate) to a staging
batch; the batch is aggregated on the GPU when it fills, before an import (so arrival order
across ProcessMetric and ImportMetric is kept) and at Flush.  Flush returns WorkerMetrics whose
samplers are views of the engine's flush results: their .Flush() builds the InterMetrics exactly
as samplers.go does, and .Export() returns the forwarded JSONMetric (the engine's device
GobEncode / MarshalBinary when Flush(forward=True) asked for it).
"""
import enum
import logging
import struct
import time
from dataclasses import dataclass, field
from typing import Dict, List, NamedTuple, Optional, Union

import numpy as np

COUNTER_TYPE, GAUGE_TYPE, HISTOGRAM_TYPE, SET_TYPE, TIMER_TYPE = "counter", "gauge", "histogram", "set", "timer"
SINK_PREFIX = "veneursinkonly:"  # samplers.go:104
log = logging.getLogger("veneur_amd.worker")


class MetricScope(enum.IntEnum):  # parser.go:30-36
    MixedScope = 0
    LocalOnly = 1
    GlobalOnly = 2


class MetricType(enum.IntEnum):  # samplers.go:17-26
    CounterMetric = 0
    GaugeMetric = 1


class Aggregate(enum.IntFlag):  # samplers.go:60-68
    AggregateMin = 1 << 0
    AggregateMax = 1 << 1
    AggregateMedian = 1 << 2
    AggregateAverage = 1 << 3
    AggregateCount = 1 << 4
    AggregateSum = 1 << 5
    AggregateHarmonicMean = 1 << 6


AGGREGATES_LOOKUP = {"min": Aggregate.AggregateMin, "max": Aggregate.AggregateMax,
                     "median": Aggregate.AggregateMedian, "avg": Aggregate.AggregateAverage,
                     "count": Aggregate.AggregateCount, "sum": Aggregate.AggregateSum,
                     "hmean": Aggregate.AggregateHarmonicMean}


@dataclass
class HistogramAggregates:  # samplers.go:80-83
    value: Aggregate = Aggregate(0)
    count: int = 0


# veneur's default (server.go:144-146): min, max, count
DEFAULT_AGGREGATES = HistogramAggregates(Aggregate.AggregateMin | Aggregate.AggregateMax | Aggregate.AggregateCount, 3)


class MetricKey(NamedTuple):  # parser.go:39-43 (comparable: the worker's map key)
    name: str
    type: str
    joined_tags: str = ""


@dataclass
class UDPMetric:  # parser.go:21-28
    key: MetricKey
    value: Union[float, str]
    sample_rate: float = 1.0
    digest: int = 0
    tags: List[str] = field(default_factory=list)
    scope: MetricScope = MetricScope.MixedScope


@dataclass
class JSONMetric:  # samplers.go:97-102
    key: MetricKey
    tags: List[str]
    value: bytes


@dataclass
class InterMetric:  # samplers.go:45-56
    name: str
    timestamp: int
    value: float
    tags: List[str]
    type: MetricType
    sinks: Optional[set] = None


def route_info(tags):
    """routeInfo (samplers.go:106-122): sinks named by veneursinkonly: tags, or None (all)."""
    info = None
    for t in tags:
        if t.startswith(SINK_PREFIX):
            info = info if info is not None else set()
            info.add(t[len(SINK_PREFIX):])
    return info


def _im(name, now, value, tags, typ, sinks):
    return InterMetric(name, now, float(value), list(tags), typ, sinks)


# ---------------------------------------------------------------- flushed samplers
@dataclass
class Counter:
    name: str
    tags: List[str]
    value: int  # int64 (samplers.go:125-129)
    key: MetricKey = None

    def flush(self, interval=None):  # samplers.go:136-147
        return [_im(self.name, int(time.time()), float(self.value), self.tags, MetricType.CounterMetric,
                    route_info(self.tags))]

    def export(self):  # samplers.go:150-165: 8-byte little-endian int64
        return JSONMetric(MetricKey(self.name, COUNTER_TYPE, ",".join(self.tags)), list(self.tags),
                          struct.pack("<q", self.value))


@dataclass
class Gauge:
    name: str
    tags: List[str]
    value: float
    key: MetricKey = None

    def flush(self):  # samplers.go:203-215
        return [_im(self.name, int(time.time()), self.value, self.tags, MetricType.GaugeMetric,
                    route_info(self.tags))]

    def export(self):  # samplers.go:218-234: 8-byte little-endian float64
        return JSONMetric(MetricKey(self.name, GAUGE_TYPE, ",".join(self.tags)), list(self.tags),
                          struct.pack("<d", self.value))


@dataclass
class Set:
    name: str
    tags: List[str]
    estimate: int      # Hll.Estimate()
    sparse: bool
    payload: Optional[bytes] = None  # MarshalBinary, when the flush forwarded it
    key: MetricKey = None

    def flush(self):  # samplers.go:282-294: the estimate as a GaugeMetric
        return [_im(self.name, int(time.time()), float(self.estimate), self.tags, MetricType.GaugeMetric,
                    route_info(self.tags))]

    def export(self):  # samplers.go:296-310
        if self.payload is None:
            raise ValueError("set %r was not exported: flush(forward=True)" % self.name)
        return JSONMetric(MetricKey(self.name, SET_TYPE, ",".join(self.tags)), list(self.tags), self.payload)


@dataclass
class Histo:
    name: str
    tags: List[str]
    local_weight: float
    local_min: float
    local_max: float
    local_sum: float
    local_reciprocal_sum: float
    quantiles: Dict[float, float]     # Value.Quantile(p) for the engine's percentiles
    payload: Optional[bytes] = None   # GobEncode, when the flush forwarded it
    type_name: str = HISTOGRAM_TYPE
    key: MetricKey = None

    def quantile(self, p):
        try:
            return self.quantiles[float(p)]
        except KeyError:
            raise ValueError("percentile %r was not computed at flush: add it to the Worker's percentiles" % p)

    def flush(self, interval, percentiles, aggregates: HistogramAggregates):  # samplers.go:373-498
        now = int(time.time())
        sinks = route_info(self.tags)
        a = Aggregate(aggregates.value)
        out = []
        G, Cm = MetricType.GaugeMetric, MetricType.CounterMetric
        inf = float("inf")
        if a & Aggregate.AggregateMax and abs(self.local_max) != inf:
            out.append(_im(self.name + ".max", now, self.local_max, self.tags, G, sinks))
        if a & Aggregate.AggregateMin and abs(self.local_min) != inf:
            out.append(_im(self.name + ".min", now, self.local_min, self.tags, G, sinks))
        if a & Aggregate.AggregateSum and self.local_sum != 0:
            out.append(_im(self.name + ".sum", now, self.local_sum, self.tags, G, sinks))
        if a & Aggregate.AggregateAverage and self.local_sum != 0 and self.local_weight != 0:
            out.append(_im(self.name + ".avg", now, self.local_sum / self.local_weight, self.tags, G, sinks))
        if a & Aggregate.AggregateCount and self.local_weight != 0:
            out.append(_im(self.name + ".count", now, self.local_weight, self.tags, Cm, sinks))
        if a & Aggregate.AggregateMedian:
            out.append(_im(self.name + ".median", now, self.quantile(0.5), self.tags, G, sinks))
        if a & Aggregate.AggregateHarmonicMean and self.local_reciprocal_sum != 0 and self.local_weight != 0:
            out.append(_im(self.name + ".hmean", now, self.local_weight / self.local_reciprocal_sum, self.tags, G,
                           sinks))
        for p in percentiles:  # "%s.%dpercentile" with int(p*100): p99.9 is named 99percentile, as in Go
            out.append(_im("%s.%dpercentile" % (self.name, int(p * 100)), now, self.quantile(p), self.tags, G, sinks))
        return out

    def export(self):  # samplers.go:501-510
        if self.payload is None:
            raise ValueError("histogram %r was not exported: flush(forward=True)" % self.name)
        return JSONMetric(MetricKey(self.name, self.type_name, ",".join(self.tags)), list(self.tags), self.payload)


# ---------------------------------------------------------------- routing (host side)
def go_bytes(s: str) -> bytes:
    """The bytes of a Go string held as str: the parser keeps invalid UTF-8 as surrogate escapes
    (veneur_amd.parser), which map back to the raw bytes Go hashes and inserts."""
    return s.encode("utf-8", "surrogateescape")


def metric_digest(key: MetricKey) -> int:
    """FNV-1a 32 of name, type and joined tags: UDPMetric.Digest (parser.go:213-304) and the
    import worker hash (http.go:77-90).  Keys route to worker Digest % len(workers)."""
    h = 0x811C9DC5
    for part in (key.name, key.type, key.joined_tags):
        for b in go_bytes(part):
            h = ((h ^ b) * 0x01000193) & 0xFFFFFFFF
    return h


def route_udp(workers, m: UDPMetric):
    """Server.HandleMetricPacket's hand-off (server.go:655): workers[Digest % n].IngestUDP."""
    d = m.digest if m.digest else metric_digest(m.key)
    workers[d % len(workers)].ingest_udp(m)


def json_metrics_by_worker(metrics, num_workers):
    """newJSONMetricsByWorker (http.go:71-139): the imported metrics ordered by worker index,
    yielded as contiguous (chunk, worker index) runs.  Go's sort.Sort leaves the order inside
    a worker's run unspecified; this keeps arrival order there (one of the orders it allows)."""
    idx = [metric_digest(m.key) % num_workers for m in metrics]
    order = sorted(range(len(metrics)), key=lambda i: idx[i])
    i = 0
    while i < len(order):
        j = i
        while j < len(order) and idx[order[j]] == idx[order[i]]:
            j += 1
        yield [metrics[k] for k in order[i:j]], idx[order[i]]
        i = j


def import_metrics(workers, metrics):
    """Server.ImportMetrics (http.go:52-67): each worker's chunk to its worker, in order -- one
    batched engine call per sampler class (Worker.import_chunk) where Go sends the chunk down the
    worker's ImportChan and ImportMetric()s it metric by metric."""
    for chunk, w in json_metrics_by_worker(metrics, len(workers)):
        workers[w].import_chunk(chunk)


# map name -> (engine class, type name); worker.go:40-58
_MAPS = {
    "counters": (0, COUNTER_TYPE), "global_counters": (0, COUNTER_TYPE),
    "gauges": (1, GAUGE_TYPE), "global_gauges": (1, GAUGE_TYPE),
    "histograms": (2, HISTOGRAM_TYPE), "local_histograms": (2, HISTOGRAM_TYPE),
    "timers": (2, TIMER_TYPE), "local_timers": (2, TIMER_TYPE),
    "sets": (3, SET_TYPE), "local_sets": (3, SET_TYPE),
}


def _map_for(typ, scope):
    """Upsert's map choice (worker.go:81-138)."""
    if typ == COUNTER_TYPE:
        return "global_counters" if scope == MetricScope.GlobalOnly else "counters"
    if typ == GAUGE_TYPE:
        return "global_gauges" if scope == MetricScope.GlobalOnly else "gauges"
    if typ == HISTOGRAM_TYPE:
        return "local_histograms" if scope == MetricScope.LocalOnly else "histograms"
    if typ == SET_TYPE:
        return "local_sets" if scope == MetricScope.LocalOnly else "sets"
    if typ == TIMER_TYPE:
        return "local_timers" if scope == MetricScope.LocalOnly else "timers"
    return None


class WorkerMetrics:
    """The flushed window: one dict MetricKey -> sampler per reference map (worker.go:40-58)."""

    def __init__(self):
        for m in _MAPS:
            setattr(self, m, {})

    def __len__(self):
        return sum(len(getattr(self, m)) for m in _MAPS)


class _Window:
    """Interned keys of one flush window: per map MetricKey -> (slot, tags); slots are dense per
    engine class (the engine resets the touched slots at flush, so every window restarts at 0)."""

    def __init__(self):
        self.maps = {m: {} for m in _MAPS}
        self.next_slot = [0, 0, 0, 0]

    def upsert(self, map_name, key, tags, cap):
        d = self.maps[map_name]
        hit = d.get(key)
        if hit is not None:
            return hit[0]
        cls = _MAPS[map_name][0]
        s = self.next_slot[cls]
        if s >= cap[cls]:
            raise OverflowError("more %s keys in one window than the engine's capacity (%d)" %
                                (("counter", "gauge", "histo", "set")[cls], cap[cls]))
        self.next_slot[cls] = s + 1
        d[key] = (s, list(tags))
        return s


class WorkerStats:
    """The two calls Worker.Flush makes on its statsd client (worker.go:286-295), recorded:
    ("timing" | "count", name, value, tags, rate) per call, in call order.  Pass any object with
    the same two methods (a statsd client) as Worker(stats=...) to send them instead."""

    def __init__(self):
        self.calls = []

    def TimeInMilliseconds(self, name, value, tags, rate):
        self.calls.append(("timing", name, float(value), tags, rate))

    def Count(self, name, value, tags, rate):
        self.calls.append(("count", name, int(value), tags, rate))


class PendingWorkerMetrics(WorkerMetrics):
    """The WorkerMetrics of a window whose engine is still flushing (Worker(pipeline=D > 1)).

    The reference's Worker.Flush only swaps the maps under the lock (worker.go:276-284); the
    flusher reads the swapped maps afterwards (flusher.go:115-230).  Here Flush hands the window's
    engine to a flush thread of its own and returns at once; the ten maps are filled the first
    time any of them is read, which waits for that engine's vn_flush."""

    def __init__(self, future):
        self._future = future

    def done(self):
        return self._future.done()

    def wait(self, timeout=None):
        """The flushed window's maps (blocks until the engine's flush has returned)."""
        if "counters" not in self.__dict__:
            wm = self._future.result(timeout)
            self.__dict__.update({m: getattr(wm, m) for m in _MAPS})
        return self

    def __getattr__(self, name):
        if name in _MAPS:
            self.wait()
            return self.__dict__[name]
        raise AttributeError(name)


class Worker:
    """veneur Worker (worker.go) whose samplers live in HBM.

    engine: a veneur_amd.Engine (or anything with its ingest/import/export/flush methods);
    created from `capacity`/`percentiles` when omitted.  percentiles: the quantiles Flush
    computes (0.5 is always added for the median aggregate).

    pipeline / engines: D engines on the GPU taking the flush windows in turn, as the
    reference's Worker.Flush swaps in fresh maps and the flusher works on the old ones while the
    worker takes the next interval (worker.go:276-284, flusher.go:115-230).  Flush() drains the
    window into the current engine, starts that engine's flush on a thread of its own and returns
    a PendingWorkerMetrics; ProcessMetric and ImportMetric move to the next engine at once.  An
    engine takes records again only after its previous flush has returned (the first call that
    needs it waits), so D windows at most are in flight.  D > 1 needs every engine stream on a
    hardware queue of its own: GPU_MAX_HW_QUEUES=16 in the environment before HIP starts
    (INTEGRATION.md); Worker sets it when it creates the engines and HIP has not started yet."""

    def __init__(self, id=0, capacity=(1 << 16, 1 << 16, 1 << 16, 1 << 16), percentiles=(0.5, 0.9, 0.99),
                 batch_records=1 << 16, engine=None, stats=None, pipeline=1, engines=None, **engine_kw):
        self.id = id
        # the worker's own statsd client (worker.go:30,286-295); a WorkerStats recorder by default
        self.stats = stats if stats is not None else WorkerStats()
        pct = tuple(sorted(set(float(p) for p in percentiles) | {0.5}))
        if engines is None:
            if engine is not None:
                if int(pipeline) > 1:
                    raise ValueError("engine= runs one engine; pass engines=[...] for pipeline > 1")
                engines = [engine]
            else:
                from .engine import Engine
                if pipeline > 1:
                    import os
                    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
                engines = [Engine(capacity, percentiles=pct, max_batch_records=max(batch_records, 1),
                                  max_batch_member_bytes=max(batch_records, 1) * 64, **engine_kw)
                           for _ in range(max(1, int(pipeline)))]
        self._engines = list(engines)
        self._cur = 0
        self._pending = [None] * len(self._engines)  # each engine's last flush (a Future), D > 1
        self._flushers = None
        if len(self._engines) > 1:
            from concurrent.futures import ThreadPoolExecutor
            self._flushers = [ThreadPoolExecutor(1, thread_name_prefix="veneur-flush-%s-%d" % (id, k))
                              for k in range(len(self._engines))]
        engine = self._engines[0]
        self.capacity = tuple(int(c) for c in getattr(engine, "capacity", capacity))
        self.percentiles = tuple(float(p) for p in getattr(engine, "percentiles", pct))
        # one ingest call carries at most the engines' max_batch_records, and of each class at most
        # its max_class_records (vn_config.max_batch_class_records): the stage drains at either
        self.batch_records = int(batch_records)
        caps = [getattr(e, "max_class_records", None) for e in self._engines]
        mbr = [int(getattr(e, "max_batch_records", 0) or 0) for e in self._engines]
        if all(mbr):
            self.batch_records = min([self.batch_records] + mbr)
        self.class_records = tuple(min([self.batch_records] + [int(c[k]) for c in caps if c]) for k in range(4))
        self.processed = 0
        self.imported = 0
        self.dropped = 0  # histogram records with a NaN sample rate (see process_metric)
        self.flush_errors = 0  # engine flushes that failed on a flush thread (D > 1, see _eng)
        # whole staged batches the engine refused (ingest raised), and their records: every value
        # the engine validates is screened in process_metric first, so these stay exceptional
        self.dropped_batches = 0
        self.dropped_batch_records = 0
        # set member bytes one ingest call may carry (the engine's max_batch_member_bytes)
        self.max_member_bytes = min(int(getattr(e, "max_batch_member_bytes", 0) or max(batch_records, 1) * 64)
                                    for e in self._engines)
        self._win = _Window()
        self._reset_stage()

    # ------------------------------------------------------------ engines in turn
    @property
    def engine(self):
        """The engine taking this window's records."""
        return self._engines[self._cur]

    @property
    def pipeline(self):
        return len(self._engines)

    def _eng(self):
        """The current engine, once its previous flush (D windows ago) has returned.  If that flush
        failed, its error is raised here (the engine's window was never flushed, so it must not
        take the next window's records on top of it) and counted in flush_errors; the engine is
        taken again only after a flush of it succeeds (the caller may call Flush again)."""
        p = self._pending[self._cur]
        if p is not None:
            from concurrent.futures import wait
            wait([p])
            self._pending[self._cur] = None
            err = p.exception()
            if err is not None:
                self.flush_errors += 1
                log.error("flush of engine %d failed: %s", self._cur, err)
                raise err
        return self._engines[self._cur]

    def _hand_off(self, job):
        """Run job (the flush of the current engine) now (D = 1) or on that engine's flush thread,
        and move ingest to the next engine (D > 1): the map swap of worker.go:276-284."""
        if self._flushers is None:
            return job()
        self._eng()
        fut = self._flushers[self._cur].submit(job)
        self._pending[self._cur] = fut
        self._cur = (self._cur + 1) % len(self._engines)
        return fut

    # ------------------------------------------------------------ staging
    def _reset_stage(self):
        self._c = ([], [], [])
        self._g = ([], [])
        self._h = ([], [], [])
        self._s = ([], [])
        self._staged = 0
        self._cls_staged = [0, 0, 0, 0]
        self._member_bytes = 0

    def _drain(self):
        """Aggregate the staged ProcessMetric records on the GPU (arrival order per class)."""
        if not self._staged:
            return
        kw = {}
        if self._c[0]:
            kw["counters"] = (np.array(self._c[0], np.uint32), np.array(self._c[1], np.float64),
                              np.array(self._c[2], np.float32))
        if self._g[0]:
            kw["gauges"] = (np.array(self._g[0], np.uint32), np.array(self._g[1], np.float64))
        if self._h[0]:
            kw["histos"] = (np.array(self._h[0], np.uint32), np.array(self._h[1], np.float64),
                            np.array(self._h[2], np.float32))
        if self._s[0]:
            mem = self._s[1]
            off = np.zeros(len(mem) + 1, np.uint32)
            off[1:] = np.cumsum([len(m) for m in mem])
            kw["sets"] = (np.array(self._s[0], np.uint32), off, np.frombuffer(b"".join(mem) or b"\0", np.uint8))
        from .engine import EngineError
        eng = self._eng()  # (a failed earlier flush of this engine is raised here, not dropped below)
        try:
            eng.ingest(**kw)
        except EngineError as err:
            # a batch the engine rejects is dropped and counted, never resubmitted: one bad batch
            # must not block every later ProcessMetric and the window's flush
            self.dropped_batches += 1
            self.dropped_batch_records += self._staged
            log.error("dropping a batch of %d staged samples: %s", self._staged, err)
        self._reset_stage()

    # ------------------------------------------------------------ the reference's operations
    def process_metric(self, m: UDPMetric):
        """Worker.ProcessMetric (worker.go:187-227)."""
        self.processed += 1
        map_name = _map_for(m.key.type, m.scope)
        if map_name is None:
            log.error("Unknown metric type for processing: %s", m.key.type)
            return
        cls = _MAPS[map_name][0]
        if cls == 3:
            if not isinstance(m.value, str):
                raise TypeError("set sample value must be a string (samplers.go:265)")
        else:
            v = float(m.value)
            if cls == 2 and (v != v or v in (float("inf"), float("-inf"))):
                raise ValueError("invalid value added")  # MergingDigest.Add panics (merging_digest.go:98-100)
        rate = np.float32(m.sample_rate)
        if cls == 2 and not (0.0 < rate <= 1.0):
            # The parser rejects rates outside (0, 1] but lets NaN through (parser.go:262-272:
            # both comparisons are false).  A counter samples any rate as Go does
            # (int64(float32(1/NaN)) = MinInt64 on amd64; the engine reproduces it).  A histogram's
            # NaN weight passes MergingDigest.Add (it checks weight <= 0), and Go's next
            # mergeAllTemps over the NaN-mean centroid that follows never terminates
            # ("NaN sample rates"; tests/test_oracle_kats.py): the engine refuses
            # such a record (VN_EINVAL), so it is dropped and counted here, one record, and the
            # rest of the batch is unaffected.
            self.dropped += 1
            log.warning("dropping %s sample with sample rate %r", m.key.name, m.sample_rate)
            return
        if cls == 3:
            member = go_bytes(m.value)
            if self._member_bytes + len(member) > self.max_member_bytes:
                self._drain()  # the engine takes at most max_batch_member_bytes per call
            if len(member) > self.max_member_bytes:
                raise ValueError("set member of %d bytes exceeds max_batch_member_bytes" % len(member))
        slot = self._win.upsert(map_name, m.key, m.tags, self.capacity)
        if cls == 0:
            self._c[0].append(slot), self._c[1].append(v), self._c[2].append(rate)
        elif cls == 1:
            self._g[0].append(slot), self._g[1].append(v)
        elif cls == 2:
            self._h[0].append(slot), self._h[1].append(v), self._h[2].append(rate)
        else:
            self._s[0].append(slot), self._s[1].append(member)
            self._member_bytes += len(member)
        self._staged += 1
        self._cls_staged[cls] += 1
        if self._staged >= self.batch_records or self._cls_staged[cls] >= self.class_records[cls]:
            self._drain()

    ProcessMetric = process_metric

    def ingest_udp(self, m: UDPMetric):
        """IngestUDP (worker.go:36-38): the channel hand-off is a direct call here."""
        self.process_metric(m)

    def import_metric(self, other: JSONMetric):
        """Worker.ImportMetric (worker.go:230-268): counters/gauges go to the global maps, sets and
        histograms/timers to the mixed-scope maps; a payload that fails to decode is logged and
        skipped, as Combine's error is."""
        self.imported += 1
        typ = other.key.type
        scope = MetricScope.GlobalOnly if typ in (COUNTER_TYPE, GAUGE_TYPE) else MetricScope.MixedScope
        map_name = _map_for(typ, scope)
        if map_name is None:
            log.error("Unknown metric type for importing: %s", typ)
            return
        slot = self._win.upsert(map_name, other.key, other.tags, self.capacity)
        self._drain()  # samples staged before this import are aggregated first
        cls = _MAPS[map_name][0]
        from .engine import EngineError
        eng = self._eng()
        try:
            # Counter/Gauge.Combine decode with binary.Read, which reads the first 8 bytes and
            # fails only on a shorter payload (samplers.go:171-183, 237-249)
            if cls == 0:
                if len(other.value) < 8:
                    raise EngineError("counter payload is %d bytes, fewer than 8" % len(other.value))
                eng.import_counters(np.array([slot], np.uint32), np.array(struct.unpack("<q", bytes(other.value[:8]))))
            elif cls == 1:
                if len(other.value) < 8:
                    raise EngineError("gauge payload is %d bytes, fewer than 8" % len(other.value))
                eng.import_gauges(np.array([slot], np.uint32), np.array(struct.unpack("<d", bytes(other.value[:8]))))
            elif cls == 2:
                eng.import_histos(np.array([slot], np.uint32), [bytes(other.value)])
            else:
                eng.import_sets(np.array([slot], np.uint32), [bytes(other.value)])
        except EngineError as err:
            log.error("Could not merge %s: %s", map_name.replace("global_", ""), err)

    ImportMetric = import_metric

    def import_chunk(self, metrics):
        """ImportMetric for every metric of a chunk (worker.go:230-268), with one engine call per
        sampler class and piece of at most that class's record cap (max_class_records): same Upsert,
        same arrival order within a class (the only order that can matter: a key belongs to one
        class), and a payload that fails to decode is logged and skipped alone -- a failing piece is
        retried metric by metric."""
        from .engine import EngineError
        groups = {0: [], 1: [], 2: [], 3: []}
        for m in metrics:
            self.imported += 1
            typ = m.key.type
            scope = MetricScope.GlobalOnly if typ in (COUNTER_TYPE, GAUGE_TYPE) else MetricScope.MixedScope
            map_name = _map_for(typ, scope)
            if map_name is None:
                log.error("Unknown metric type for importing: %s", typ)
                continue
            slot = self._win.upsert(map_name, m.key, m.tags, self.capacity)
            cls = _MAPS[map_name][0]
            if cls in (0, 1) and len(m.value) < 8:
                log.error("Could not merge %s: payload is %d bytes, fewer than 8", map_name.replace("global_", ""),
                          len(m.value))
                continue
            groups[cls].append((slot, m, map_name))
        self._drain()  # samples staged before the chunk are aggregated first
        eng = self._eng()
        for cls in (0, 1, 2, 3):
            items = groups[cls]
            cap = max(1, self.class_records[cls])
            for i in range(0, len(items), cap):
                piece = items[i:i + cap]
                slots = np.array([g[0] for g in piece], np.uint32)
                if cls == 0:
                    eng.import_counters(slots, np.array([struct.unpack("<q", bytes(g[1].value[:8]))[0] for g in piece],
                                                        np.int64))
                    continue
                if cls == 1:
                    eng.import_gauges(slots, np.array([struct.unpack("<d", bytes(g[1].value[:8]))[0] for g in piece],
                                                      np.float64))
                    continue
                fn = eng.import_histos if cls == 2 else eng.import_sets
                try:
                    fn(slots, [bytes(g[1].value) for g in piece])
                except EngineError:  # find the bad payload(s): the engine applied nothing of the piece
                    for slot, m, map_name in piece:
                        try:
                            fn(np.array([slot], np.uint32), [bytes(m.value)])
                        except EngineError as err:
                            log.error("Could not merge %s: %s", map_name, err)

    def process_batch(self, batch=None, **arrays):
        """A batch of ProcessMetric calls whose keys the caller has interned itself -- the cgo
        binding's path (Go fills the engine's pinned stage, vn_submit) or the device
        intake's: an A.Batch whose arrays are in device memory (vn_ingest), or host arrays as
        Engine.ingest takes them (counters=(slot, value, rate), gauges=, histos=, sets= or
        set_hashes=; arrival order per class).  Those keys have no MetricKey on the host, so they
        appear in flush_raw()'s result, not in Flush()'s maps."""
        self._drain()
        if batch is not None:
            self._eng().ingest_device(batch)
            self.processed += int(batch.n_counter + batch.n_gauge + batch.n_histo + batch.n_set)
        else:
            self._eng().ingest(**arrays)
            self.processed += sum(len(v[0]) for v in arrays.values())

    def flush(self, forward=False, is_local=False, need_median=False) -> WorkerMetrics:
        """Worker.Flush (worker.go:271-298): the window's samplers, and a fresh window.  With
        forward=True the mixed-scope histograms/timers and sets are also exported (GobEncode /
        MarshalBinary on the GPU) for flushForward (flusher.go:264-353).  is_local: this is a
        local veneur, whose Server.Flush asks no percentiles of mixed-scope histograms/timers
        and flushes no mixed-scope sets (flusher.go:41-48,181-211) -- the engine then skips
        those quantiles and estimates (vn_flush_masked); need_median keeps the quantiles, as
        Histo.Flush evaluates Quantile(0.5) for the median aggregate regardless.

        With D > 1 engines (pipeline) the engine's flush runs on its flush thread and this
        returns a PendingWorkerMetrics at once (the class docstring)."""
        start = time.perf_counter_ns()
        self._drain()
        win = self._take_window()
        eng = self._eng()

        def job():
            payload = {}
            if forward:
                for cls, names, fn in ((2, ("histograms", "timers"), eng.export_histos),
                                       (3, ("sets",), eng.export_sets)):
                    slots = [s for n in names for (s, _) in win.maps[n].values()]
                    if slots:
                        for s, p in zip(slots, fn(np.array(slots, np.uint32))):
                            payload[(cls, s)] = p
            if is_local:
                qmask, emask = self._masks(win, need_median)
                f = eng.flush(histo_quantile_mask=qmask, set_estimate_mask=emask)
            else:
                f = eng.flush()
            return self._worker_metrics(win, f, payload)

        out = self._hand_off(job)
        self._flush_stats(start)
        return out if self._flushers is None else PendingWorkerMetrics(out)

    def flush_raw(self, histo_quantile_mask=None, set_estimate_mask=None, copy=False):
        """Worker.Flush returning the engine's flush result itself (per class: touched slots and
        their values, histogram stats and quantiles, set estimates) instead of the ten maps: for
        callers that interned their keys themselves (process_batch).  copy=False: the
        vn_flush_result, whose arrays live in the engine's pinned memory until that engine's next
        flush (D windows later); copy=True: a FlushOutput of numpy copies.  With D > 1 engines it
        returns a concurrent.futures.Future of the result."""
        start = time.perf_counter_ns()
        self._drain()
        self._take_window()
        eng = self._eng()

        def job():
            return (eng.flush if copy else eng.flush_raw)(histo_quantile_mask, set_estimate_mask)

        out = self._hand_off(job)
        self._flush_stats(start)
        return out

    def _flush_stats(self, start):
        """The end of Worker.Flush (worker.go:286-295): reset processed/imported and report the
        flush's duration and the window's counts through the worker's statsd client."""
        processed, imported = self.processed, self.imported
        self.processed = 0
        self.imported = 0
        self.stats.TimeInMilliseconds("flush.worker_duration_ns", float(time.perf_counter_ns() - start), None, 1.0)
        self.stats.Count("worker.metrics_processed_total", processed, [], 1.0)
        self.stats.Count("worker.metrics_imported_total", imported, [], 1.0)

    def _take_window(self):
        """The map swap of Worker.Flush (worker.go:277-284): the window's interned keys, and a
        fresh window."""
        win, self._win = self._win, _Window()
        return win

    def _masks(self, win, need_median):
        qmask = np.zeros(self.capacity[2], np.uint8)
        emask = np.zeros(self.capacity[3], np.uint8)
        for names, mask, on in ((("local_histograms", "local_timers"), qmask, 1),
                                (("histograms", "timers"), qmask, 1 if need_median else 0),
                                (("local_sets",), emask, 1), (("sets",), emask, 0)):
            for n in names:
                for s_, _ in win.maps[n].values():
                    mask[s_] = on
        return qmask, emask

    def flush_datadog(self, sink, histogram_percentiles, aggregates: "HistogramAggregates" = None, is_local=False,
                      timestamp=None):
        """Worker.Flush, then the window's InterMetrics straight into the Datadog sink's request
        bodies (veneur_amd.sink, vn_datadog_flush): generateInterMetrics (flusher.go:168-230) +
        finalizeMetrics and chunking (sinks/datadog/datadog.go:77-106,160-213) + PostHelper's JSON
        (http/http.go:116-135) in C++, with no per-key Python objects.  Returns ([(ok, body)],
        (n_intermetrics, n_metrics)); with D > 1 engines, a concurrent.futures.Future of it."""
        aggregates = aggregates or DEFAULT_AGGREGATES
        start = time.perf_counter_ns()
        self._drain()
        win = self._take_window()
        eng = self._eng()

        def job():
            if is_local:
                qm, em = self._masks(win, bool(Aggregate(aggregates.value) & Aggregate.AggregateMedian))
                f = eng.flush_raw(histo_quantile_mask=qm, set_estimate_mask=em)
            else:
                f = eng.flush_raw()
            return sink.bodies(f, win.maps, self.percentiles, histogram_percentiles, aggregates, is_local, timestamp)

        out = self._hand_off(job)
        self._flush_stats(start)
        return out

    def _worker_metrics(self, win, f, payload):
        by_cls = [dict(zip(f.counter_slot.tolist(), f.counter_value.tolist())),
                  dict(zip(f.gauge_slot.tolist(), f.gauge_value.tolist())),
                  {int(s): i for i, s in enumerate(f.histo_slot)},
                  {int(s): i for i, s in enumerate(f.set_slot)}]
        wm = WorkerMetrics()
        for map_name, (cls, typ) in _MAPS.items():
            out = getattr(wm, map_name)
            for key, (s, tags) in win.maps[map_name].items():
                if cls == 0:
                    out[key] = Counter(key.name, tags, int(by_cls[0].get(s, 0)), key)
                elif cls == 1:
                    out[key] = Gauge(key.name, tags, float(by_cls[1].get(s, 0.0)), key)
                elif cls == 2:
                    i = by_cls[2].get(s)
                    if i is None:  # upserted by an import that failed to decode: an empty Histo
                        st = [0.0, float("inf"), float("-inf"), 0.0, 0.0]
                        q = {p: float("nan") for p in self.percentiles}
                    else:
                        st = f.histo_stats[i].tolist()
                        q = dict(zip(self.percentiles, f.histo_quantiles[i].tolist()))
                    out[key] = Histo(key.name, tags, st[0], st[1], st[2], st[3], st[4], q, payload.get((2, s)), typ,
                                     key)
                else:
                    i = by_cls[3].get(s)
                    est = int(f.set_estimate[i]) if i is not None else 0
                    sparse = bool(f.set_sparse[i]) if i is not None else True
                    out[key] = Set(key.name, tags, est, sparse, payload.get((3, s)), key)
        return wm

    Flush = flush

    def wait(self):
        """Wait for every engine's pending flush (D > 1)."""
        from concurrent.futures import wait
        wait([p for p in self._pending if p is not None])

    def close(self, close_engines=True):
        if self._flushers is not None:
            self.wait()
            for x in self._flushers:
                x.shutdown(wait=True)
            self._flushers = None
        if close_engines:
            for e in self._engines:
                if hasattr(e, "close"):
                    e.close()


# ---------------------------------------------------------------- Server.Flush (metrics part)
def generate_inter_metrics(wms, percentiles, histogram_percentiles, aggregates: HistogramAggregates, is_local,
                           interval=10.0) -> List[InterMetric]:
    """generateInterMetrics (flusher.go:168-230): every WorkerMetrics' samplers flushed in the
    reference's map order.  percentiles is nil on a local veneur (mixed histograms and timers get
    only their local aggregates); local-only histograms/timers always use histogram_percentiles;
    mixed sets, global counters and global gauges are flushed by a global veneur only (a local
    one forwards them)."""
    out = []
    for wm in wms:
        for c in wm.counters.values():
            out += c.flush(interval)
        for g in wm.gauges.values():
            out += g.flush()
        for h in wm.histograms.values():
            out += h.flush(interval, percentiles, aggregates)
        for t in wm.timers.values():
            out += t.flush(interval, percentiles, aggregates)
        for h in wm.local_histograms.values():
            out += h.flush(interval, histogram_percentiles, aggregates)
        for s in wm.local_sets.values():
            out += s.flush()
        for t in wm.local_timers.values():
            out += t.flush(interval, histogram_percentiles, aggregates)
        if not is_local:
            for s in wm.sets.values():
                out += s.flush()
            for gc in wm.global_counters.values():
                out += gc.flush(interval)
            for gg in wm.global_gauges.values():
                out += gg.flush()
    return out


def server_flush(workers, is_local, histogram_percentiles, aggregates: HistogramAggregates = DEFAULT_AGGREGATES,
                 interval=10.0):
    """Server.Flush's metric path (flusher.go:18-92; events, traces, sinks and plugins are out of
    scope): tallyMetrics flushes every worker (115-163), generateInterMetrics builds the
    InterMetrics, and a local veneur also returns flushForward's JSONMetrics for its global
    (264-353; POSTing them is http_import.post_body's job).  Returns (InterMetrics, forwarded)."""
    from .http_import import flush_forward
    percentiles = [] if is_local else list(histogram_percentiles)  # flusher.go:41-48
    need_median = bool(Aggregate(aggregates.value) & Aggregate.AggregateMedian)
    wms = [w.flush(forward=is_local, is_local=is_local, need_median=need_median) for w in workers]
    final = generate_inter_metrics(wms, percentiles, histogram_percentiles, aggregates, is_local, interval)
    return final, (flush_forward(wms) if is_local else [])
