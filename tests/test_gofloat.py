"""CPU checks of the device parser's ParseFloat (veneur_amd/csrc/gofloat.h, run on the host
through vn_go_parse_float): Go 1.9 strconv.ParseFloat(s, 64 | 32) syntax and correctly rounded
values (samplers/parser.go:239,261), against glibc strtod / strtof -- correctly rounded, so any
correct decimal conversion must agree bit for bit -- on hard cases (halfway points, subnormal and
overflow boundaries, more than 19 digits, far exponents) and on random decimal strings."""
import ctypes as C
import math
import random
import re
import struct

import pytest

GO_SYNTAX = re.compile(rb"^[+-]?([0-9]+(\.[0-9]*)?|\.[0-9]+)([eE][+-]?[0-9]+)?$")
SPECIAL = re.compile(rb"^([+-]?(inf|infinity)|nan)$", re.I)


@pytest.fixture(scope="module")
def libs():
    import veneur_amd._abi as A
    libc = C.CDLL(None)
    libc.strtod.restype = C.c_double
    libc.strtod.argtypes = [C.c_char_p, C.POINTER(C.c_char_p)]
    libc.strtof.restype = C.c_float
    libc.strtof.argtypes = [C.c_char_p, C.POINTER(C.c_char_p)]
    return A, libc


def go_parse(A, s, bits):
    out = C.c_double()
    rc = A.lib.vn_go_parse_float(s, len(s), bits, C.byref(out))
    return rc, out.value


def f64bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def expected(libc, s, bits):
    """Go's answer via glibc: (status, value) with status 0 ok, 1 syntax, 2 range."""
    if SPECIAL.match(s):
        low = s.lower().lstrip(b"+-")
        if low == b"nan":
            return 0, math.nan
        return 0, -math.inf if s.startswith(b"-") else math.inf
    if not GO_SYNTAX.match(s):
        return 1, None
    v = float(libc.strtof(s, None)) if bits == 32 else libc.strtod(s, None)
    if math.isinf(v):
        return 2, None
    return 0, v


def check(A, libc, s, bits):
    rc, v = go_parse(A, s, bits)
    erc, ev = expected(libc, s, bits)
    assert rc == erc, (s, bits, rc, erc)
    if rc == 0:
        if math.isnan(ev):
            assert math.isnan(v), s
        else:
            assert f64bits(v) == f64bits(ev), (s, bits, v.hex(), ev.hex())


HARD = [
    b"0", b"-0", b"+0", b"0.0", b"-0.000e5", b".5", b"5.", b"1e0", b"1E+2", b"1e-2", b"+1.5", b"00012.500",
    b"9007199254740993", b"9007199254740992", b"9007199254740994", b"9007199254740995",
    b"4503599627370497", b"4503599627370496.5", b"4503599627370497.5",
    b"1.00000000000000011102230246251565404236316680908203125",   # halfway 1 .. 1+ulp
    b"1.00000000000000011102230246251565404236316680908203124",
    b"1.00000000000000011102230246251565404236316680908203126",
    b"2.4703282292062327e-324", b"2.4703282292062328e-324", b"4.9406564584124654e-324", b"5e-324", b"1e-400",
    b"2.2250738585072011e-308", b"2.2250738585072012e-308", b"2.2250738585072014e-308",
    b"1.7976931348623157e308", b"1.7976931348623158e308", b"1.7976931348623159e308", b"1e309", b"-1e309",
    b"179769313486231580793728971405301e276",
    b"0.1", b"0.2", b"0.3", b"123456789012345678901234567890", b"1234567890123456789", b"12345678901234567890",
    b"1.2345678901234567890123", b"49.53118934218371", b"0.000000000000000000000000000001",
    b"1e23", b"8.41e21", b"5e-20", b"3.0e-27", b"9.999999999999999e22", b"1e22", b"1e-22", b"123e-25",
    b"1" + b"0" * 400, b"0." + b"0" * 400 + b"1", b"1" * 800 + b"e-700", b"7" * 900,
    b"1.00000005960464477539062500", b"1.00000005960464477539062499", b"1.00000005960464477539062501",
    b"3.4028235e38", b"3.40282356779733661637539395458142568448e38", b"3.4028236e38", b"1e39",
    b"1.4e-45", b"7.006492321624085e-46", b"7.006492321624086e-46", b"1e-46", b"1.17549435e-38",
    b"0.5", b"0.25", b"0.1", b"1", b"1.0", b"0.333333333", b"16777217", b"16777216.5", b"33554435",
    b"inf", b"-Inf", b"+INFINITY", b"nan", b"NaN", b"-nan", b"infinit", b"in", b"",
    b"1e", b"1e+", b".", b"-", b"+.e1", b"1..2", b"1.2.3", b"0x10", b"1_000", b" 1", b"1 ", b"1e5x", b"e5",
    b"1e10000", b"1e-10000", b"1e99999999999", b"-1e-99999999999",
]


@pytest.mark.parametrize("bits", [64, 32])
def test_hard_cases(libs, bits):
    A, libc = libs
    for s in HARD:
        check(A, libc, s, bits)


def rand_decimal(rng):
    sign = rng.choice([b"", b"-", b"+"])
    nd = rng.choice([1, 2, 3, 5, 8, 12, 15, 16, 17, 18, 19, 20, 21, 25, 30, 40])
    digits = bytes(rng.choice(b"0123456789") for _ in range(nd))
    if rng.random() < 0.3:
        digits = digits.lstrip(b"0") or b"0"
    mode = rng.random()
    if mode < 0.4:
        cut = rng.randint(0, len(digits))
        m = digits[:cut] + b"." + digits[cut:]
        if m == b".":
            m = b"0."
    else:
        m = digits
    if rng.random() < 0.6:
        e = rng.choice([rng.randint(-30, 30), rng.randint(-340, 320), rng.randint(-60, 60)])
        m += rng.choice([b"e", b"E"]) + (b"+" if e >= 0 and rng.random() < 0.3 else b"") + str(e).encode()
    return sign + m


def halfway(rng, bits):
    """Decimal strings at or next to the exact midpoint between two adjacent floats."""
    from decimal import Decimal, getcontext
    getcontext().prec = 1200
    if bits == 64:
        x = struct.unpack("<d", struct.pack("<Q", rng.randrange(1, 0x7FEFFFFFFFFFFFFF)))[0]
        nx = math.nextafter(x, math.inf)
    else:
        u = rng.randrange(1, 0x7F7FFFFF)
        x = struct.unpack("<f", struct.pack("<I", u))[0]
        nx = struct.unpack("<f", struct.pack("<I", u + 1))[0]
    mid = (Decimal(x) + Decimal(nx)) / 2
    s = format(mid, "e").encode()
    out = [s]
    mant, _, exp = s.partition(b"e")
    if b"." in mant and len(mant) > 20:  # nudge the last digit
        for d in (b"1", b"9"):
            out.append(mant[:-1] + d + b"e" + exp)
        out.append(mant[:20] + b"e" + exp)
    return out


@pytest.mark.parametrize("bits", [64, 32])
def test_random_decimals(libs, bits):
    A, libc = libs
    rng = random.Random(1009 + bits)
    for _ in range(60000):
        check(A, libc, rand_decimal(rng), bits)


@pytest.mark.parametrize("bits", [64, 32])
def test_halfway_points(libs, bits):
    A, libc = libs
    rng = random.Random(77 + bits)
    for _ in range(3000):
        for s in halfway(rng, bits):
            check(A, libc, s, bits)


def test_random_doubles_roundtrip(libs):
    A, libc = libs
    rng = random.Random(5)
    for _ in range(50000):
        x = struct.unpack("<d", struct.pack("<Q", rng.randrange(0, 0x7FF0000000000000)))[0]
        for s in (repr(x).encode(), ("%.17g" % x).encode(), ("%.15g" % x).encode(), ("%.25e" % x).encode()):
            check(A, libc, s, 64)
            check(A, libc, s, 32)
