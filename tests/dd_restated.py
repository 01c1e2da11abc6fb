"""Test infrastructure: the Datadog sink's flush restated in Python, the checker of the native
vn_datadog_flush (csrc/sink.cpp).

  finalize_metrics   sinks/datadog/datadog.go:160-213 (IsAcceptableMetric, sinks/sinks.go:32-37)
  chunks             datadog.go:77-106 (rounding-up division under flushMaxPerBody)
  encode_body        json.NewEncoder(w).Encode(map[string][]DDMetric{"series": chunk})
                     (http/http.go:116-135, datadog.go:215-218): DDMetric field order and
                     omitempty (datadog.go:41-49), Go 1.8+ float encoding (ES6 cut-offs, shortest
                     digits, "e-07" -> "e-7"), HTML-escaped strings; NaN / Inf -> unsupported value
InterMetrics come from veneur_amd.worker.generate_inter_metrics (flusher.go:168-230) over the
WorkerMetrics of Worker.Flush, with their timestamps replaced by one fixed value.
"""
import math
from decimal import Decimal

from veneur_amd.http_import import _go_json_string
from veneur_amd.worker import MetricType


class Unsupported(ValueError):
    pass


def go_json_float(f):
    """encoding/json floatEncoder for float64 (Go 1.8+)."""
    if math.isnan(f) or math.isinf(f):
        raise Unsupported("json: unsupported value: %r" % f)
    if f == 0:
        return "-0" if math.copysign(1.0, f) < 0 else "0"
    f = float(f)
    t = Decimal(repr(f)).as_tuple()  # shortest round-trip digits (repr is correctly rounded)
    digits = list(t.digits)
    exp = t.exponent
    while len(digits) > 1 and digits[-1] == 0:
        digits.pop()
        exp += 1
    m = "".join(map(str, digits))
    x = exp + len(m) - 1  # value = m[0].m[1:] * 10^x
    sign = "-" if t.sign else ""
    a = abs(f)
    if a < 1e-6 or a >= 1e21:
        s = m[0] + ("." + m[1:] if len(m) > 1 else "") + "e" + ("-" if x < 0 else "+") + "%02d" % abs(x)
        if x < 0 and abs(x) < 10:
            s = s[:-2] + s[-1]  # e-07 -> e-7
        return sign + s
    dp = x + 1
    if dp <= 0:
        return sign + "0." + "0" * (-dp) + m
    if dp >= len(m):
        return sign + m + "0" * (dp - len(m))
    return sign + m[:dp] + "." + m[dp:]


def finalize_metrics(ims, interval, hostname, sink_tags):
    """finalizeMetrics: DDMetric dicts (ordered as DDMetric's fields)."""
    out = []
    for m in ims:
        if m.sinks is not None and "datadog" not in m.sinks:
            continue
        value = m.value / interval if m.type == MetricType.CounterMetric else m.value
        dd = {"metric": m.name, "points": [[float(m.timestamp), value]], "tags": list(sink_tags),
              "type": "rate" if m.type == MetricType.CounterMetric else "gauge", "host": "", "device_name": "",
              "interval": int(interval)}
        for t in m.tags:
            if t.startswith("host:"):
                dd["host"] = t[5:]
            elif t.startswith("device:"):
                dd["device_name"] = t[7:]
            else:
                dd["tags"].append(t)
        if dd["host"] == "":
            dd["host"] = hostname
        out.append(dd)
    return out


def chunks(metrics, max_per_body):
    n = len(metrics)
    workers = (n - 1) // max_per_body + 1 if n else 1  # Go's -1 / k == 0
    size = (n - 1) // workers + 1 if n else 0
    return [metrics[i * size:] if i == workers - 1 else metrics[i * size:(i + 1) * size] for i in range(workers)]


def encode_body(chunk):
    """(ok, bytes): the encoder's output, or (False, b"") when a value cannot be encoded."""
    try:
        objs = []
        for d in chunk:
            s = '{"metric":' + _go_json_string(d["metric"])
            s += ',"points":[[' + go_json_float(d["points"][0][0]) + "," + go_json_float(d["points"][0][1]) + "]]"
            if d["tags"]:
                s += ',"tags":[' + ",".join(_go_json_string(t) for t in d["tags"]) + "]"
            s += ',"type":' + _go_json_string(d["type"])
            if d["host"]:
                s += ',"host":' + _go_json_string(d["host"])
            if d["device_name"]:
                s += ',"device_name":' + _go_json_string(d["device_name"])
            if d["interval"]:
                s += ',"interval":%d' % d["interval"]
            objs.append(s + "}")
    except Unsupported:
        return False, b""
    return True, ('{"series":[' + ",".join(objs) + "]}\n").encode("utf-8", "surrogateescape")


def datadog_bodies(ims, interval, hostname, sink_tags, max_per_body, timestamp):
    for m in ims:
        m.timestamp = timestamp
    fin = finalize_metrics(ims, interval, hostname, sink_tags)
    return [encode_body(c) for c in chunks(fin, max_per_body)], (len(ims), len(fin))
