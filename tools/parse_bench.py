#!/usr/bin/env python3
"""Throughput of the device DogStatsD parse (vn_parse_dogstatsd_device) on a buffer already in HBM,
beside the host parse (vn_parse_dogstatsd, one core) of the same buffer.

Lines look like a C4 stream: 1M keys, Zipf key choice, DogStatsD types in the C3 mix, 3 tags
(unsorted) per line, 10% sampled.  Prints one JSON line.
    python tools/parse_bench.py [--lines 4000000] [--reps 10]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_buffer(n, seed=7, n_keys=1_000_000):
    rng = np.random.default_rng(seed)
    keys = rng.zipf(1.3, n) % n_keys
    kind = keys % 20
    out = []
    for i in range(n):
        k = int(keys[i])
        c = int(kind[i])
        if c < 8:
            v, t = b"%d" % (1 + (i % 10)), b"c"
        elif c < 12:
            v, t = b"%.2f" % ((i * 7919) % 100000 / 100.0), b"g"
        elif c < 17:
            v, t = b"%.3f" % (1.0 + (i * 104729) % 500000 / 1000.0), b"ms"
        else:
            v, t = b"u%d" % (i % 50000), b"s"
        rate = b"|@0.5" if i % 10 == 0 else b""
        out.append(b"svc.metric.%d:%s|%s%s|#zone:z%d,env:prod,host:h%d" % (k, v, t, rate, k % 7, k % 101))
    return b"\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=4_000_000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import veneur_amd._abi as A
    from veneur_amd.intake import DeviceParser, parse_host
    buf = make_buffer(a.lines)
    with DeviceParser(max_bytes=len(buf) + 1, max_lines=a.lines + 1) as p:
        A.lib.vn_copy_to_device(0, p.buf.ptr, C.c_char_p(buf), len(buf))
        n = p.parse_resident(len(buf))  # warm-up
        A.lib.vn_device_synchronize(0)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            p.parse_resident(len(buf))
        A.lib.vn_device_synchronize(0)
        dt = (time.perf_counter() - t0) / a.reps
    sample = buf[: len(buf) // 8]
    sample = sample[: sample.rfind(b"\n")]
    t0 = time.perf_counter()
    hl, _ = parse_host(sample)
    ht = time.perf_counter() - t0
    print(json.dumps({"kernel": "vn_parse_dogstatsd_device", "lines": n, "bytes": len(buf),
                      "ms_per_buffer": dt * 1e3, "lines_per_s": n / dt, "GBs": len(buf) / dt / 1e9,
                      "host_lines_per_s_1core": len(hl) / ht, "host_sample_lines": len(hl)}))


if __name__ == "__main__":
    main()
