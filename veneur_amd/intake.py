"""DogStatsD text on the GPU: the device parse (vn_parse_dogstatsd_device, csrc/parse_device.hip).

The reference parses every UDP packet on the host (samplers/parser.go:186-307 ParseMetric, called
per '\n'-separated line by server.go:693-722) before Worker.ProcessMetric; here a whole buffer of
datagram lines already in HBM is parsed by the GPU, with the host parse (vn_parse_dogstatsd) as
its checker.  DeviceParser owns the parser handle and the device buffers it fills.
"""
import ctypes as C

import numpy as np

from . import _abi as A

PARSED_DTYPE = np.dtype([("line_off", "<u8"), ("name_off", "<u8"), ("value_off", "<u8"), ("tags_off", "<u8"),
                         ("value", "<f8"), ("line_len", "<u4"), ("name_len", "<u4"), ("value_len", "<u4"),
                         ("tags_len", "<u4"), ("n_tags", "<u4"), ("digest", "<u4"), ("rate", "<f4"),
                         ("status", "<i4"), ("type", "u1"), ("scope", "u1"), ("has_tags", "u1"), ("pad", "u1"),
                         ("_align", "<u4")])
assert PARSED_DTYPE.itemsize == C.sizeof(A.ParsedLine)


class DeviceError(RuntimeError):
    pass


class _Dev:
    """A device allocation (vn_device_alloc) freed with its owner."""

    def __init__(self, device, nbytes):
        self.ptr = C.c_void_p()
        self.nbytes = int(nbytes)
        rc = A.lib.vn_device_alloc(device, max(1, self.nbytes), C.byref(self.ptr))
        if rc != 0:
            raise DeviceError("vn_device_alloc(%d) failed (%d)" % (self.nbytes, rc))

    def free(self):
        if self.ptr:
            A.lib.vn_device_free(self.ptr)
            self.ptr = C.c_void_p()


class DeviceParser:
    """vn_parser: parses datagram buffers of up to max_bytes bytes / max_lines lines on `device`."""

    def __init__(self, max_bytes=1 << 24, max_lines=1 << 20, device=0):
        self.device, self.max_bytes, self.max_lines = device, int(max_bytes), int(max_lines)
        self.h = C.c_void_p()
        rc = A.lib.vn_parser_create(device, self.max_bytes, self.max_lines, C.byref(self.h))
        if rc != 0:
            raise DeviceError("vn_parser_create failed (%d)" % rc)
        self.buf = _Dev(device, self.max_bytes)
        self.tags = _Dev(device, self.max_bytes)
        self.out = _Dev(device, self.max_lines * PARSED_DTYPE.itemsize)

    def close(self):
        for b in (self.buf, self.tags, self.out):
            b.free()
        if self.h:
            A.lib.vn_parser_destroy(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def parse_resident(self, nbytes):
        """Parse the first nbytes of self.buf (already in HBM); returns the line count."""
        n = C.c_uint64()
        rc = A.lib.vn_parse_dogstatsd_device(self.h, self.buf.ptr, nbytes, self.out.ptr, self.max_lines, self.tags.ptr,
                                             self.max_bytes, C.byref(n))
        if rc != 0:
            raise DeviceError("vn_parse_dogstatsd_device: %s (%d)" %
                              (A.lib.vn_parser_last_error(self.h).decode(errors="replace"), rc))
        return n.value

    def parse(self, datagram: bytes):
        """Copy a datagram buffer to HBM and parse it: (lines as a PARSED_DTYPE array, tags_out bytes)."""
        if len(datagram) > self.max_bytes:
            raise ValueError("buffer of %d bytes exceeds max_bytes" % len(datagram))
        if datagram:
            A.lib.vn_copy_to_device(self.device, self.buf.ptr, C.c_char_p(datagram), len(datagram))
        n = self.parse_resident(len(datagram))
        lines = np.zeros(n, PARSED_DTYPE)
        tags = np.zeros(max(1, len(datagram)), np.uint8)
        if n:
            A.lib.vn_copy_to_host(self.device, lines.ctypes.data_as(C.c_void_p), self.out.ptr, n * PARSED_DTYPE.itemsize)
            A.lib.vn_copy_to_host(self.device, tags.ctypes.data_as(C.c_void_p), self.tags.ptr, len(tags))
        return lines, tags.tobytes()[:len(datagram)]


def parse_host(datagram: bytes, max_lines=None):
    """vn_parse_dogstatsd (host C++) with the same output layout: the checker of the device parse."""
    max_lines = max_lines if max_lines is not None else datagram.count(b"\n") + 1
    lines = np.zeros(max(1, max_lines), PARSED_DTYPE)
    tags = C.create_string_buffer(max(1, len(datagram)))
    n = A.lib.vn_parse_dogstatsd(datagram, len(datagram), lines.ctypes.data_as(C.POINTER(A.ParsedLine)), max_lines,
                                 tags, max(1, len(datagram)))
    if n < 0:
        raise ValueError("vn_parse_dogstatsd failed (%d)" % n)
    return lines[:n], tags.raw[:len(datagram)]


# ---------------------------------------------------------------- Worker on the device intake
_MAP_IDS = ("counters", "global_counters", "gauges", "global_gauges", "histograms", "local_histograms", "timers",
            "local_timers", "sets", "local_sets")
_MAP_TYPE = ("counter", "counter", "gauge", "gauge", "histogram", "histogram", "timer", "timer", "set", "set")


class _DeviceWindow:
    """The window's interned keys, held by the device key table (vn_intake): upsert() is the
    host-side Upsert (ImportMetric, ProcessMetric of a host UDPMetric) and `maps` reads the table
    back as the host Worker's _Window layout, map name -> {MetricKey: (slot, tags)}."""

    def __init__(self, intake):
        self.intake = intake

    def upsert(self, map_name, key, tags, cap):
        from .worker import go_bytes, metric_digest
        name, jt = go_bytes(key.name), go_bytes(key.joined_tags)
        blob = name + jt
        arr = lambda v, t: np.array(v, t)
        slot = np.zeros(1, np.uint32)
        h = self.intake.h
        rc = A.lib.vn_intake_upsert(
            h, 1, arr([_MAP_IDS.index(map_name)], np.uint8).ctypes.data_as(A.u8p),
            arr([len(tags)], np.uint32).ctypes.data_as(A.u32p), arr([metric_digest(key)], np.uint32).ctypes.data_as(A.u32p),
            arr([0], np.uint32).ctypes.data_as(A.u32p), arr([len(name)], np.uint32).ctypes.data_as(A.u32p),
            arr([len(name)], np.uint32).ctypes.data_as(A.u32p), arr([len(jt)], np.uint32).ctypes.data_as(A.u32p),
            C.cast(C.c_char_p(blob or b"\0"), A.u8p), len(blob), slot.ctypes.data_as(A.u32p))
        if rc != 0:
            msg = A.lib.vn_intake_last_error(h).decode(errors="replace")
            if "capacity" in msg:
                raise OverflowError(msg)
            raise DeviceError("vn_intake_upsert: %s (%d)" % (msg, rc))
        return int(slot[0])

    @property
    def maps(self):
        from .worker import MetricKey
        info = A.IntakeInfo()
        A.lib.vn_intake_keys_info(self.intake.h, C.byref(info))
        k = int(info.n_keys)
        mp, slot, nt = np.zeros(k, np.uint8), np.zeros(k, np.uint32), np.zeros(k, np.uint32)
        noff, nlen, tlen = np.zeros(k, np.uint64), np.zeros(k, np.uint32), np.zeros(k, np.uint32)
        arena = np.zeros(max(1, int(info.arena_bytes)), np.uint8)
        rc = A.lib.vn_intake_read_keys(self.intake.h, mp.ctypes.data_as(A.u8p), slot.ctypes.data_as(A.u32p),
                                       nt.ctypes.data_as(A.u32p), noff.ctypes.data_as(A.u64p),
                                       nlen.ctypes.data_as(A.u32p), tlen.ctypes.data_as(A.u32p),
                                       arena.ctypes.data_as(A.u8p))
        if rc != 0:
            raise DeviceError("vn_intake_read_keys failed (%d)" % rc)
        raw = arena.tobytes()
        out = {m: {} for m in _MAP_IDS}
        for i in range(k):
            o, n, t = int(noff[i]), int(nlen[i]), int(tlen[i])
            name = raw[o:o + n].decode("utf-8", "surrogateescape")
            jt = raw[o + n:o + n + t].decode("utf-8", "surrogateescape")
            tags = jt.split(",") if nt[i] else []
            out[_MAP_IDS[mp[i]]][MetricKey(name, _MAP_TYPE[mp[i]], jt)] = (int(slot[i]), tags)
        return out


class Intake:
    """vn_intake over an Engine: DogStatsD datagram buffers -> ProcessMetric on the GPU."""

    def __init__(self, engine, max_bytes=1 << 24, max_lines=None):
        self.engine = engine
        self.max_bytes = int(max_bytes)
        self.max_lines = int(max_lines or min(min(engine.max_class_records), max(1, self.max_bytes // 4)))
        self.h = C.c_void_p()
        rc = A.lib.vn_intake_create(engine.h, self.max_bytes, self.max_lines, C.byref(self.h))
        if rc != 0:
            raise DeviceError("vn_intake_create failed (%d)" % rc)
        self.buf = _Dev(engine.device, self.max_bytes)

    def process_resident(self, nbytes):
        """vn_intake_process of the first nbytes of self.buf (already in HBM)."""
        st = A.IntakeStats()
        rc = A.lib.vn_intake_process(self.h, self.buf.ptr, nbytes, C.byref(st))
        if rc != 0:
            msg = A.lib.vn_intake_last_error(self.h).decode(errors="replace")
            if "capacity" in msg:
                raise OverflowError(msg)
            raise DeviceError("vn_intake_process: %s (%d)" % (msg, rc))
        return {f: int(getattr(st, f)) for f, _ in A.IntakeStats._fields_}

    def process(self, datagram: bytes):
        if len(datagram) > self.max_bytes:
            raise ValueError("buffer of %d bytes exceeds max_bytes" % len(datagram))
        if datagram:
            A.lib.vn_copy_to_device(self.engine.device, self.buf.ptr, C.c_char_p(datagram), len(datagram))
        return self.process_resident(len(datagram))

    def reset(self):
        if A.lib.vn_intake_reset(self.h) != 0:
            raise DeviceError("vn_intake_reset failed")

    def close(self):
        self.buf.free()
        if self.h:
            A.lib.vn_intake_destroy(self.h)
            self.h = C.c_void_p()


def DeviceWorker(*args, intake_bytes=1 << 24, **kw):
    """A veneur Worker (worker.py) whose ProcessMetric path takes DogStatsD text on the GPU:
    handle_packets(datagram) = ReadMetricSocket's loop over a buffer of '\\n'-separated packets
    (server.go:693-722) -> ParseMetric -> ProcessMetric, parse and Upsert on the device.  Imports and
    host UDPMetrics intern through the same device key table, so every path shares the slots."""
    from .worker import Worker, _Window

    class _DeviceWorker(Worker):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            if self.pipeline > 1:
                # the device key table lives beside one engine, and Flush reads it back at once
                raise ValueError("DeviceWorker drives one engine (pipeline=1)")
            self.intake = Intake(self.engine, intake_bytes)
            self._win = _DeviceWindow(self.intake)
            self.parse_errors = 0

        def handle_packets(self, datagram: bytes):
            self._drain()  # host-staged records come first
            st = self.intake.process(datagram)
            self.processed += st["processed"] + st["dropped"]  # ProcessMetric counts both (worker.go:190)
            self.dropped += st["dropped"]
            self.parse_errors += st["parse_errors"]
            return st

        def _take_window(self):
            win = _Window()
            win.maps = self._win.maps  # read back from the device key table
            self.intake.reset()
            return win

        def close(self):
            self.intake.close()
            super().close()

    return _DeviceWorker(*args, **kw)
