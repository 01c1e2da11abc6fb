"""GPU parity of the device DogStatsD parse (csrc/parse_device.hip) with the host parse
vn_parse_dogstatsd (csrc/parse.cpp, itself checked line by line against the Python mirror of
samplers/parser.go:186-307 in test_parser.py): every line's status, and for the lines that parse
every field (offsets, value and rate bits, type, scope, tag count, digest) and the joined tags
byte for byte -- on the reference's parser_test.go cases, the 4000 mutated lines of
test_parser.py, and a generated 200k-line buffer with the hard number formats (17-digit values,
more than 19 digits, far exponents, long sample rates that take the decimal slow path), scope
tags, duplicate and empty tags, and empty lines."""
import numpy as np
import pytest

from tests.test_parser import INVALID, _mutations

FIELDS = ("line_off", "line_len", "name_off", "name_len", "value_off", "value_len", "type", "scope", "has_tags",
          "n_tags", "digest", "tags_off", "tags_len")


def compare(datagram, dev_parser):
    from veneur_amd.intake import parse_host
    hl, ht = parse_host(datagram)
    dl, dt = dev_parser.parse(datagram)
    assert len(dl) == len(hl)
    assert np.array_equal(dl["status"], hl["status"]), np.nonzero(dl["status"] != hl["status"])[0][:10]
    ok = hl["status"] == 0
    for f in FIELDS:
        bad = np.nonzero(dl[f][ok] != hl[f][ok])[0]
        assert len(bad) == 0, (f, [(datagram[int(hl["line_off"][ok][i]):][:80], dl[f][ok][i], hl[f][ok][i])
                                   for i in bad[:5]])
    assert np.array_equal(dl["value"][ok].view(np.uint64), hl["value"][ok].view(np.uint64))
    assert np.array_equal(dl["rate"][ok].view(np.uint32), hl["rate"][ok].view(np.uint32))
    total = int((hl["tags_len"][ok]).sum())
    assert dt[:total] == ht[:total]
    return hl


def gen_lines(rng, n):
    names = [b"svc.req", b"api.latency", b"a", b"db.q\xc3\xa9", b"x" * 40, b"m:n"]
    vals = [lambda: b"%d" % rng.integers(-5, 1000), lambda: b"%.3f" % rng.lognormal(3, 1),
            lambda: repr(float(rng.lognormal(3, 2))).encode(), lambda: b"%.17g" % rng.random(),
            lambda: b"1234567890123456789012.5", lambda: b"0.%s" % (b"9" * 25),
            lambda: b"%de-%d" % (rng.integers(1, 99), rng.integers(290, 330)), lambda: b"1e%d" % rng.integers(300, 320),
            lambda: b"-0", lambda: b"inf", lambda: b"12a", lambda: b"", lambda: b"4.5e+2"]
    types = [b"c", b"g", b"h", b"ms", b"s", b"x", b""]
    rates = [b"", b"|@0.5", b"|@0.1", b"|@1", b"|@0.1000000000000000055511151231257827", b"|@nan", b"|@2",
             b"|@1e-50", b"|@0.33333333333333333333333", b"|@", b"|@0.5|@0.5"]
    tag_pool = [b"env:prod", b"zone:a", b"veneurlocalonly", b"veneurglobalonly", b"veneurglobalonly:true", b"",
                b"env:dev", b"host:h1", b"a,b", b"veneurlocalonly:x", b"zz"]
    out = []
    for _ in range(n):
        name = names[int(rng.integers(0, len(names)))]
        t = types[int(rng.integers(0, len(types)))] if rng.random() < 0.2 else [b"c", b"g", b"h", b"ms", b"s"][
            int(rng.integers(0, 5))]
        v = b"m%d" % rng.integers(0, 1000) if t == b"s" else vals[int(rng.integers(0, len(vals)))]()
        line = name + b":" + v + b"|" + t
        if rng.random() < 0.5:
            line += rates[int(rng.integers(0, len(rates)))]
        if rng.random() < 0.7:
            k = int(rng.integers(0, 7))
            line += b"|#" + b",".join(tag_pool[int(i)] for i in rng.integers(0, len(tag_pool), k))
            if rng.random() < 0.05:
                line += b"|#dup"
        if rng.random() < 0.03:
            line += b"|@0.5"
        out.append(line)
        if rng.random() < 0.05:
            out.append(b"")
    return out


@pytest.fixture(scope="module")
def dev_parser():
    from veneur_amd.intake import DeviceParser
    with DeviceParser(max_bytes=1 << 26, max_lines=1 << 21) as p:
        yield p


@pytest.mark.gpu
def test_device_parse_reference_cases(dev_parser):
    base = [b"a.b.c:1|c", b"a.b.c:1|g", b"a.b.c:1|h", b"a.b.c:1|ms", b"a.b.c:foo|s", b"a.b.c:1|c|#foo:bar,baz:gorch",
            b"a.b.c:1|c|@0.1", b"a.b.c:1|g|@0.1", b"a.b.c:1|c|@0.1|#foo:bar,baz:gorch",
            b"a.b.c:1|h|#veneurlocalonly,tag2:quacks", b"a.b.c:1|h|#veneurglobalonly,tag2:quacks",
            b"a:1|c|#veneurlocalonly,veneurglobalonly", b"foo:1|h|#bar", b"_e{5,4}:title|text", b"_sc|x|0"]
    compare(b"\n".join(list(INVALID) + base), dev_parser)


@pytest.mark.gpu
def test_device_parse_mutations(dev_parser):
    rng = np.random.default_rng(3)
    lines = _mutations(rng, 4000)  # these may hold '\n' themselves: more, shorter lines
    compare(b"\n".join(lines), dev_parser)
    compare(b"\n\n" + b"\n".join(lines) + b"\n", dev_parser)


@pytest.mark.gpu
def test_device_parse_generated(dev_parser):
    rng = np.random.default_rng(11)
    hl = compare(b"\n".join(gen_lines(rng, 200_000)), dev_parser)
    st = hl["status"]
    assert (st == 0).sum() > 50_000 and len(set(st.tolist())) >= 8  # many parse, most error kinds occur


@pytest.mark.gpu
def test_device_parse_unaligned_buffer(dev_parser):
    """A datagram buffer that starts at an odd device address (byte loads instead of vector loads)."""
    import ctypes as C
    import veneur_amd._abi as A
    from veneur_amd.intake import PARSED_DTYPE, parse_host
    rng = np.random.default_rng(5)
    d = b"\n".join(gen_lines(rng, 3000))
    A.lib.vn_copy_to_device(0, C.c_void_p(dev_parser.buf.ptr.value + 3), C.c_char_p(d), len(d))
    n = C.c_uint64()
    assert A.lib.vn_parse_dogstatsd_device(dev_parser.h, C.c_void_p(dev_parser.buf.ptr.value + 3), len(d),
                                           dev_parser.out.ptr, dev_parser.max_lines, dev_parser.tags.ptr,
                                           dev_parser.max_bytes, C.byref(n)) == 0
    hl, _ = parse_host(d)
    dl = np.zeros(n.value, PARSED_DTYPE)
    A.lib.vn_copy_to_host(0, dl.ctypes.data_as(C.c_void_p), dev_parser.out.ptr, n.value * PARSED_DTYPE.itemsize)
    assert len(dl) == len(hl) and np.array_equal(dl["status"], hl["status"])
    ok = hl["status"] == 0
    assert np.array_equal(dl["digest"][ok], hl["digest"][ok]) and np.array_equal(dl["line_off"], hl["line_off"])


@pytest.mark.gpu
def test_device_parse_edges(dev_parser):
    long_lines = b"\n".join(b"k%d:1.5|ms|#z:%d,a:" % (i, i) + b"t" * 90 for i in range(600))  # > 16 KiB per block
    for buf in (b"", b"\n", b"\n\n\n", b"a:1|c", b"a:1|c\n", b"\na:1|c", b"x" * 5000, b"a:1|c|#" + b"t," * 2000 + b"t",
                long_lines):
        compare(buf, dev_parser)
    from veneur_amd.intake import DeviceError
    with pytest.raises(DeviceError):  # more lines than max_lines
        from veneur_amd.intake import DeviceParser
        with DeviceParser(max_bytes=1 << 10, max_lines=4) as p:
            p.parse(b"a:1|c\n" * 5)
