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
