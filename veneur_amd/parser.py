"""DogStatsD text -> UDPMetric in front of Worker.ProcessMetric (host side).

Restates the reference's metric-packet parse so that text read from the listeners reaches the
engine with the same keys, values, sample rates, scopes and routing digests:

  samplers/parser.go:186-307   ParseMetric: name:value|type[|@rate][|#tags]
  samplers/split_bytes.go      SplitBytes (bytes.IndexByte splitting, a trailing empty chunk)
  server.go:612-660            HandleMetricPacket: empty packet ignored, "_e{" / "_sc" are events
                               and service checks (not on this path), metrics to
                               Workers[Digest % len(Workers)]
  server.go:693-722            ReadMetricSocket: one datagram = metric lines joined by '\\n'

Go rules kept: the value is strconv.ParseFloat(s, 64) with Go 1.9's syntax (no underscores, no
hex floats, no surrounding spaces; "inf"/"infinity"/"nan" parse and are then rejected), the rate
is ParseFloat(s, 32) -- decimal rounded ONCE to float32 (not via float64), overflow is an error,
NaN passes the (0, 1] check as in Go -- tags are split on ',', sorted as bytes, the first tag
starting with veneurlocalonly / veneurglobalonly is removed and sets the scope, and Digest is
FNV-1a-32 over name, type name and the joined tags.  Names and tags are bytes in Go; invalid
UTF-8 survives here as surrogate escapes, and the digest is taken over the original bytes.
"""
import math
import re
from fractions import Fraction
from typing import List, Optional

import numpy as np

from .worker import MetricKey, MetricScope, UDPMetric

_TYPES = {ord("c"): "counter", ord("g"): "gauge", ord("h"): "histogram", ord("m"): "timer", ord("s"): "set"}
_DEC = re.compile(rb"[+-]?(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?")
_SPECIAL = re.compile(rb"(?i:[+-]?inf(?:inity)?|nan)")


class ParseError(ValueError):
    """ParseMetric's error; the message carries the reference's text."""


def _fnv1a(h, data: bytes):
    for b in data:
        h = ((h ^ b) * 0x01000193) & 0xFFFFFFFF
    return h


def _special(s: bytes) -> float:
    t = s.lower().lstrip(b"+")
    return float("nan") if t == b"nan" else (-math.inf if t.startswith(b"-") else math.inf)


def go_parse_float64(s: bytes) -> float:
    """strconv.ParseFloat(s, 64) (Go 1.9): correctly rounded decimal; ±Inf on overflow is an
    error; the special words parse (callers reject NaN/Inf)."""
    if _SPECIAL.fullmatch(s) and not s.lower().startswith((b"+nan", b"-nan")):
        return _special(s)
    if not _DEC.fullmatch(s):
        raise ParseError("invalid syntax")
    v = float(s)  # Python's float() is correctly rounded for this syntax
    if math.isinf(v):
        raise ParseError("value out of range")
    return v


_F32_MAX = Fraction((2 ** 24 - 1) * 2 ** 104)


def go_parse_float32(s: bytes) -> np.float32:
    """strconv.ParseFloat(s, 32): the decimal rounded once, to nearest even, to float32."""
    if _SPECIAL.fullmatch(s) and not s.lower().startswith((b"+nan", b"-nan")):
        return np.float32(_special(s))
    if not _DEC.fullmatch(s):
        raise ParseError("invalid syntax")
    mant, _, ex = s.lower().partition(b"e")
    digits = mant.lstrip(b"+-").replace(b".", b"").lstrip(b"0")
    if not digits:
        return np.float32(-0.0 if s[:1] == b"-" else 0.0)
    # the decimal's magnitude: keep Fraction away from absurd exponents (1e-99999999)
    ip, _, fp = mant.lstrip(b"+-").partition(b".")
    ip = ip.lstrip(b"0")
    ex = ex.lstrip(b"+")
    if len(ex.lstrip(b"-")) > 9:
        mag = -10 ** 9 if ex.startswith(b"-") else 10 ** 9
    else:
        mag = int(ex or b"0") + (len(ip) if ip else -(len(fp) - len(fp.lstrip(b"0"))))
    if mag > 60:
        raise ParseError("value out of range")
    if mag < -60:
        return np.float32(-0.0 if s[:1] == b"-" else 0.0)
    x = Fraction(s.decode())
    neg, x = x < 0, abs(x)
    if x == 0:
        return np.float32(-0.0 if neg else 0.0)
    e = x.numerator.bit_length() - x.denominator.bit_length()
    while Fraction(2) ** e > x:
        e -= 1
    while Fraction(2) ** (e + 1) <= x:
        e += 1
    q = max(e - 23, -149)  # ulp exponent: 24-bit significand, subnormals below 2^-126
    m = x / Fraction(2) ** q
    r = m.numerator // m.denominator
    rem = m - r
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and r % 2 == 1):
        r += 1
    v = Fraction(r) * Fraction(2) ** q
    if v > _F32_MAX:
        raise ParseError("value out of range")
    f = np.float32(float(v))  # exact: v is a float32 value
    return -f if neg else f


def parse_metric(packet: bytes) -> UDPMetric:
    """ParseMetric (samplers/parser.go:186-307)."""
    chunks = packet.split(b"|")  # SplitBytes yields exactly these chunks, in order
    first = chunks[0]
    colon = first.find(b":")
    if colon == -1:
        raise ParseError("Invalid metric packet, need at least 1 colon")
    name, value = first[:colon], first[colon + 1:]
    if not name:
        raise ParseError("Invalid metric packet, name cannot be empty")
    if len(chunks) < 2:
        raise ParseError("Invalid metric packet, need at least 1 pipe for type")
    tchunk = chunks[1]
    if not tchunk:
        raise ParseError("Invalid metric packet, metric type not specified")
    typ = _TYPES.get(tchunk[0])
    if typ is None:
        raise ParseError("Invalid type for metric")
    h = _fnv1a(_fnv1a(0x811C9DC5, name), typ.encode())
    if typ == "set":
        val = value.decode("utf-8", "surrogateescape")
    else:
        try:
            val = go_parse_float64(value)
        except ParseError:
            val = None
        if val is None or math.isnan(val) or math.isinf(val):
            raise ParseError("Invalid number for metric value: %s" % value.decode("utf-8", "replace"))
    rate, tags, joined, scope, found_rate = np.float32(1.0), None, b"", MetricScope.MixedScope, False
    for c in chunks[2:]:
        if not c:
            raise ParseError("Invalid metric packet, empty string after/between pipes")
        if c[:1] == b"@":
            if found_rate:
                raise ParseError("Invalid metric packet, multiple sample rates specified")
            try:
                sr = go_parse_float32(c[1:])
            except ParseError:
                raise ParseError("Invalid float for sample rate: %s" % c[1:].decode("utf-8", "replace"))
            if sr <= 0 or sr > 1:
                raise ParseError("Sample rate %f must be >0 and <=1" % float(sr))
            rate, found_rate = sr, True
        elif c[:1] == b"#":
            if tags is not None:
                raise ParseError("Invalid metric packet, multiple tag sections specified")
            tags = sorted(c[1:].split(b","))
            for i, t in enumerate(tags):
                if t.startswith(b"veneurlocalonly"):
                    del tags[i]
                    scope = MetricScope.LocalOnly
                    break
                if t.startswith(b"veneurglobalonly"):
                    del tags[i]
                    scope = MetricScope.GlobalOnly
                    break
            joined = b",".join(tags)
            h = _fnv1a(h, joined)
        else:
            raise ParseError("Invalid metric packet, contains unknown section %r" % c.decode("utf-8", "replace"))
    dec = lambda b: b.decode("utf-8", "surrogateescape")  # noqa: E731
    return UDPMetric(MetricKey(dec(name), typ, dec(joined)), val, rate, digest=h,
                     tags=[dec(t) for t in tags] if tags is not None else [], scope=scope)


ParseMetric = parse_metric


def handle_metric_packet(workers, packet: bytes) -> Optional[UDPMetric]:
    """HandleMetricPacket (server.go:612-660) for metric lines: parse, then
    Workers[Digest % len(Workers)].ProcessMetric.  Events and service checks ("_e{", "_sc")
    belong to the EventWorker, outside the aggregation path: they are rejected here."""
    if not packet:
        return None
    if packet.startswith((b"_e{", b"_sc")):
        raise ParseError("events and service checks are not handled by the aggregation path")
    m = parse_metric(packet)
    workers[m.digest % len(workers)].process_metric(m)
    return m


def read_metric_datagram(workers, datagram: bytes) -> List[Exception]:
    """ReadMetricSocket's per-datagram loop (server.go:706-714): each '\\n'-separated packet to
    handle_metric_packet; a packet that fails to parse is counted and skipped (the returned
    errors), as packet.error_total is in Go."""
    errs = []
    for p in datagram.split(b"\n"):
        try:
            handle_metric_packet(workers, p)
        except ParseError as e:
            errs.append(e)
    return errs


_NTYPES = ("counter", "gauge", "histogram", "timer", "set")


def parse_datagram_native(datagram: bytes):
    """vn_parse_dogstatsd (veneur_amd/csrc/parse.cpp): the C-ABI parse of a whole datagram.
    Returns one entry per non-empty line: a UDPMetric, or the VN_PARSE_* error code (int)."""
    import ctypes as C

    from . import _abi as A
    n_max = datagram.count(b"\n") + 1
    out = (A.ParsedLine * n_max)()
    tags = C.create_string_buffer(len(datagram) + 1)
    n = A.lib.vn_parse_dogstatsd(datagram, len(datagram), out, n_max, tags, len(datagram) + 1)
    if n < 0:
        raise ParseError("vn_parse_dogstatsd failed (%d)" % n)
    res, tb = [], tags.raw
    dec = lambda b: b.decode("utf-8", "surrogateescape")  # noqa: E731
    for o in out[:n]:
        if o.status:
            res.append(int(o.status))
            continue
        typ = _NTYPES[o.type]
        name = datagram[o.name_off:o.name_off + o.name_len]
        joined = tb[o.tags_off:o.tags_off + o.tags_len]
        val = dec(datagram[o.value_off:o.value_off + o.value_len]) if typ == "set" else o.value
        tl = [dec(t) for t in joined.split(b",")] if o.has_tags and o.n_tags else []
        res.append(UDPMetric(MetricKey(dec(name), typ, dec(joined)), val, np.float32(o.rate), digest=o.digest,
                             tags=tl, scope=MetricScope(o.scope)))
    return res
