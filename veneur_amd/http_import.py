"""veneur's POST /import envelope in front of the engine's import path.

A local veneur forwards its mixed histograms/timers, sets and global counters/gauges to the
global veneur as one JSON array of JSONMetric, optionally zlib-deflated.  This module restates
the request side of that hand-off so a global built on the engine accepts the same bodies and
answers them with the same status codes:

  handlers_global.go:53-63    handleImport: decode, then ImportMetrics (asynchronously in Go)
  handlers_global.go:110-188  unmarshalMetricsFromHTTP: Content-Encoding "" / "deflate" / other,
                              json.Decoder into []samplers.JSONMetric, empty-list check
  handlers_global.go:192-206  nonEmpty: at least one element differs from the zero JSONMetric
  http.go:52-67               Server.ImportMetrics -> workers' ImportMetric (worker.import_metrics)
  samplers/parser.go:39-43, samplers/samplers.go:97-102   the JSON field names

The payloads inside (gob t-digests, axiomhq HLL binaries, LE int64/f64) are decoded and merged
on the GPU by Worker.import_metric -> Engine.import_* (DESIGN.md §7); this layer only turns the
HTTP body into JSONMetric objects.  It is host code by nature (zlib + JSON text), like the Go
handler it mirrors.

Go decoding rules kept here:
  * the body is read as ONE JSON value; anything after it is ignored (json.Decoder.Decode);
  * field names match case-insensitively (encoding/json's fold), unknown fields are ignored,
    a JSON null leaves the field at its zero value, the last duplicate key wins;
  * a field of the wrong JSON type, invalid base64 in "value", NaN/Infinity literals, or a top
    level that is neither an array nor null is a decode error (400, cause:json);
  * "deflate" is zlib: a bad 2-byte header or a preset dictionary fails zlib.NewReader (400,
    cause:deflate); a stream that breaks later is an error only if the JSON value is not
    complete in the bytes inflated before the break (the decoder scans its buffer before it
    looks at the read error) -- the adler32 trailer is never reached in that case either;
  * Go's nil vs empty distinction matters to nonEmpty: "tags": [] and "value": "" are non-empty.
"""
import base64
import binascii
import json
import re
import logging
import zlib
from typing import List, Optional, Tuple

from .engine import EngineError
from .worker import JSONMetric, MetricKey, import_metrics

log = logging.getLogger("veneur_amd.http_import")

StatusAccepted = 202
StatusBadRequest = 400
StatusUnsupportedMediaType = 415

# encoding/json field names of samplers.JSONMetric (MetricKey embedded, so promoted)
_FIELDS = ("name", "type", "tagstring", "tags", "value")


class ImportRequestError(ValueError):
    """An /import body that unmarshalMetricsFromHTTP rejects; .status is the HTTP code and .cause
    the import.request_error_total cause tag (None where Go emits no counter)."""

    def __init__(self, status, msg, cause=None):
        super().__init__(msg)
        self.status, self.cause = status, cause


def _fold(s: str) -> str:
    """encoding/json's key folding for these ASCII field names: ASCII case, plus the two
    non-ASCII runes that fold to 's' and 'k' (U+017F, U+212A) -- fold.go's equalFoldRight."""
    return s.replace("\u017f", "s").replace("\u212a", "k").lower()


def _zlib_inflate(body: bytes) -> bytes:
    """compress/zlib.NewReader + reads until the stream ends or breaks: returns every byte
    inflated before the break.  Header errors raise (they fail NewReader itself)."""
    if len(body) < 2:
        raise ImportRequestError(StatusBadRequest, "unexpected EOF", "deflate")
    cmf, flg = body[0], body[1]
    if (cmf & 0x0F) != 8 or ((cmf << 8) | flg) % 31 != 0:
        raise ImportRequestError(StatusBadRequest, "zlib: invalid header", "deflate")
    if flg & 0x20:  # FDICT with no dictionary supplied
        raise ImportRequestError(StatusBadRequest, "zlib: invalid dictionary", "deflate")
    d = zlib.decompressobj(-15)  # raw deflate after the header; the trailer is not consulted
    out, pos, step = [], 2, 1 << 16
    while pos < len(body) and not d.eof:
        chunk = body[pos:pos + step]
        saved = d.copy()
        try:
            out.append(d.decompress(chunk))
            pos += len(chunk)
        except zlib.error:
            # keep what inflates before the break: redo this chunk one byte at a time
            d = saved
            for i in range(len(chunk)):
                try:
                    out.append(d.decompress(chunk[i:i + 1]))
                except zlib.error:
                    return b"".join(out)
            return b"".join(out)
    if not d.eof:
        try:
            out.append(d.flush())
        except zlib.error:
            pass
    return b"".join(out)


def _reject_constant(name):
    raise ValueError("invalid character '%s' looking for beginning of value" % name[0])


_DECODER = json.JSONDecoder(parse_constant=_reject_constant)


def _first_value(text: bytes):
    """json.Decoder.Decode: one value after optional whitespace; trailing bytes ignored."""
    s = text.decode("utf-8", errors="replace")  # Go substitutes U+FFFD for invalid UTF-8
    i = len(s) - len(s.lstrip(" \t\r\n"))
    if i == len(s):
        raise ValueError("EOF")
    val, _ = _DECODER.raw_decode(s, i)
    return val


def _go_bytes(v):
    """[]byte from a JSON string: base64.StdEncoding (padding required; '\\r' and '\\n' skipped)."""
    try:
        return base64.b64decode(v.replace("\r", "").replace("\n", ""), validate=True)
    except (binascii.Error, ValueError) as e:
        raise ValueError("illegal base64 data: %s" % e)


_LONE_SURROGATE = re.compile("[\ud800-\udfff]")


def _go_str(v: str) -> str:
    """Go's JSON decoder turns an escaped lone surrogate (\\ud800 not followed by its pair) into
    U+FFFD; Python's keeps it, and it cannot be encoded as UTF-8 (pairs arrive combined)."""
    return _LONE_SURROGATE.sub("\ufffd", v)


def _decode_metric(obj) -> Optional[dict]:
    """One element of []samplers.JSONMetric; None stands for Go's zero value fields."""
    m = {"name": "", "type": "", "tagstring": "", "tags": None, "value": None}
    if obj is None:
        return m
    if not isinstance(obj, dict):
        raise ValueError("json: cannot unmarshal %s into Go value of type samplers.JSONMetric"
                         % type(obj).__name__)
    err = None
    for k, v in obj.items():  # document order: the last duplicate wins
        f = _fold(k)
        if f not in _FIELDS or v is None:
            continue
        if f in ("name", "type", "tagstring"):
            if isinstance(v, str):
                m[f] = _go_str(v)
            else:
                err = err or "json: cannot unmarshal into Go struct field .%s of type string" % f
        elif f == "tags":
            if isinstance(v, list) and all(t is None or isinstance(t, str) for t in v):
                m[f] = ["" if t is None else _go_str(t) for t in v]
            else:
                err = err or "json: cannot unmarshal into Go struct field .tags of type []string"
        else:
            if isinstance(v, str):
                m[f] = _go_bytes(v)
            else:
                err = err or "json: cannot unmarshal into Go struct field .value of type []uint8"
    if err:  # Go finishes the value, then reports the first type error
        raise ValueError(err)
    return m


def _non_empty(raw: List[dict]) -> bool:
    """nonEmpty (handlers_global.go:192-206): reflect.DeepEqual against JSONMetric{}."""
    zero = {"name": "", "type": "", "tagstring": "", "tags": None, "value": None}
    return any(m != zero for m in raw)


def unmarshal_metrics_from_http(body: bytes, content_encoding: str = "") -> List[JSONMetric]:
    """unmarshalMetricsFromHTTP (handlers_global.go:110-188): the JSONMetrics of one /import
    body, or ImportRequestError with the status code the Go handler writes."""
    if content_encoding == "":
        text = body
    elif content_encoding == "deflate":
        text = _zlib_inflate(body)
    else:
        raise ImportRequestError(StatusUnsupportedMediaType, content_encoding, "unknown_content_encoding")
    try:
        top = _first_value(text)
        if top is not None and not isinstance(top, list):
            raise ValueError("json: cannot unmarshal %s into Go value of type []samplers.JSONMetric"
                             % type(top).__name__)
        raw = [_decode_metric(o) for o in (top or [])]
    except ValueError as e:
        raise ImportRequestError(StatusBadRequest, str(e), "json")
    if not raw:
        raise ImportRequestError(StatusBadRequest, "Received empty /import request")
    if not _non_empty(raw):
        raise ImportRequestError(StatusBadRequest, "Received empty or improperly-formed metrics")
    return [JSONMetric(MetricKey(m["name"], m["type"], m["tagstring"]), list(m["tags"] or []),
                       m["value"] if m["value"] is not None else b"") for m in raw]


UnmarshalMetricsFromHTTP = unmarshal_metrics_from_http


def handle_import(workers, body: bytes, content_encoding: str = "", shard=None) -> Tuple[int, int]:
    """handleImport (handlers_global.go:53-63) for a POST /import: returns (HTTP status, number
    of metrics handed to the workers).  Go runs ImportMetrics in a goroutine after answering
    202; here it runs before returning, so a caller sees the merge done on the device.

    shard=(rank, world): a global veneur spread over `world` GPUs, one process each, every
    process handed the same bodies -- this rank imports only the keys it owns (digest % world,
    dist.route_imports), so no imported key spans ranks and the import needs no collective.  The
    count returned is then this rank's share."""
    try:
        metrics = unmarshal_metrics_from_http(body, content_encoding)
    except ImportRequestError as e:
        log.error("Could not decode /import request (%s): %s", e.cause or "empty", e)
        return e.status, 0
    if shard is not None:
        from .dist import route_imports
        metrics = route_imports(metrics, *shard)
    import_metrics(workers, metrics)
    return StatusAccepted, len(metrics)


HandleImport = handle_import


def handle_import_routed(workers, router, body: Optional[bytes] = None, content_encoding: str = "") -> Tuple[int, int]:
    """handleImport for a global veneur over N GPUs with one decode per body: the router's source
    rank decodes the body and sends every rank its digest % N chunk (dist.ImportRouter); each rank
    imports its chunk into its workers.  Every rank calls this for every body (the source with the
    body, the others with None); returns (HTTP status, metrics imported on this rank)."""
    status, mine = router.route(body, content_encoding)
    if status == StatusAccepted and mine:
        import_metrics(workers, mine)
    return status, len(mine)


# ------------------------------------------------------------------ the local side: forwarding
def _go_json_string(s: str) -> str:
    """encoding/json's string encoder with HTML escaping (Go 1.9 encode.go: control bytes as
    \\u00xx except \\n \\r \\t; <, >, & and U+2028/2029 escaped; other runes raw UTF-8)."""
    out = ['"']
    for ch in s:
        c = ord(ch)
        if ch in '"\\':
            out.append("\\" + ch)
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif c < 0x20 or ch in "<>&" or c in (0x2028, 0x2029):
            out.append("\\u%04x" % c)
        elif 0xD800 <= c <= 0xDFFF:  # a lone surrogate is not valid UTF-8: Go writes the \ufffd escape
            out.append("\\ufffd")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def marshal_json_metrics(metrics: List[JSONMetric]) -> bytes:
    """json.NewEncoder(w).Encode([]samplers.JSONMetric) (http/http.go:127-135): field order
    name, type, tagstring, tags, value; empty tags as null (the parser leaves them nil);
    value as standard base64; one trailing newline."""
    parts = []
    for m in metrics:
        tags = "null" if not m.tags else "[" + ",".join(_go_json_string(t) for t in m.tags) + "]"
        value = "null" if m.value is None else '"%s"' % base64.b64encode(bytes(m.value)).decode()
        parts.append('{"name":%s,"type":%s,"tagstring":%s,"tags":%s,"value":%s}' % (
            _go_json_string(m.key.name), _go_json_string(m.key.type), _go_json_string(m.key.joined_tags),
            tags, value))
    return ("[" + ",".join(parts) + "]\n").encode("utf-8")


def post_body(metrics: List[JSONMetric], compress: bool = True) -> Tuple[bytes, str]:
    """PostHelper's request body and Content-Encoding (http/http.go:116-170): the JSON through a
    zlib writer when compress (flushForward always compresses, flusher.go:350)."""
    raw = marshal_json_metrics(metrics)
    return (zlib.compress(raw), "deflate") if compress else (raw, "")


def flush_forward(wms) -> List[JSONMetric]:
    """flushForward's export loop (flusher.go:264-346): per WorkerMetrics, the Export() of its
    global counters, global gauges, histograms, sets and timers, in that order (Go walks each
    map in random order; this keeps insertion order).  Samplers whose Export fails are logged
    and skipped.  The histogram/set payloads are the engine's device GobEncode / MarshalBinary,
    so the Worker must have been flushed with forward=True."""
    out = []
    for wm in wms:
        for name in ("global_counters", "global_gauges", "histograms", "sets", "timers"):
            for key, s in getattr(wm, name).items():
                try:
                    out.append(s.export())
                except EngineError as err:  # Go logs an Export error and continues
                    log.error("Could not export metric %s (%s): %s", key.name, name, err)
    return out
