"""CPU: the CSV ingest's numeric core (spatialflink_amd/csrc/gf_decimal.hpp -- the same code the
GPU parse kernel runs, built here for the host by tests/native/decimal_core.cpp) against Python's
correctly rounded float() (David Gay's algorithm) on random literals of every shape, plus Java
Double.valueOf / Long.valueOf grammar cases (FloatingDecimal.readJavaFormatString)."""
import ctypes as C
import math
import os
import random
import struct
import subprocess
from fractions import Fraction

import numpy as np
import pytest

from conftest import NATIVE_FLAGS, ROOT

OK, BAD, UNSUP = 0, 1, 2


@pytest.fixture(scope="module")
def core(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("core") / "decimal_core.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", *NATIVE_FLAGS,
                    os.path.join(ROOT, "tests", "native", "decimal_core.cpp"), "-o", out], check=True)
    L = C.CDLL(out)
    L.core_parse_double.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_double)]
    L.core_parse_long.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
    L.core_parse_many.argtypes = [C.c_char_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    return L


def parse_many(core, strs):
    b = [s.encode() for s in strs]
    off = np.zeros(len(b) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in b])
    buf = b"".join(b)
    out = np.zeros(len(b)); st = np.zeros(len(b), np.int32)
    core.core_parse_many(buf, off.ctypes.data, len(b), out.ctypes.data, st.ctypes.data)
    return out, st


def bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def check(core, strs, allow_unsupported=False):
    out, st = parse_many(core, strs)
    n_unsup = 0
    for s, v, t in zip(strs, out, st):
        if t == UNSUP and allow_unsupported:
            n_unsup += 1
            continue
        assert t == OK, s
        e = float(s.rstrip("fFdD"))
        assert bits(v) == bits(e) or (math.isnan(v) and math.isnan(e)), (s, v, e)
    return n_unsup


def test_shortest_repr_round_trip(core):
    rng = np.random.default_rng(1)
    vals = list(rng.uniform(115.5, 117.6, 50_000)) + list(rng.uniform(39.6, 41.1, 50_000))
    raw = rng.integers(0, 2**63 - 2**52 * 2047, 50_000, dtype=np.int64).view(np.float64)  # finite, any magnitude
    vals += [float(v) for v in raw if math.isfinite(v)]
    strs = [repr(float(v)) for v in vals] + ["-" + repr(float(v)) for v in vals[:1000]]
    assert check(core, strs) == 0


def test_random_decimal_literals(core):
    r = random.Random(7)
    strs = []
    for _ in range(60_000):
        nd = r.randint(1, 19)
        digits = "".join(r.choice("0123456789") for _ in range(nd))
        dot = r.randint(0, nd)
        s = digits[:dot] + "." + digits[dot:] if r.random() < 0.7 else digits
        if s == ".":
            s = "0."
        if r.random() < 0.6:
            s += r.choice("eE") + r.choice(["", "+", "-"]) + str(r.randint(0, 340))
        if r.random() < 0.3:
            s = "-" + s
        strs.append(s)
    assert check(core, strs) == 0


def test_long_significands(core):
    """> 19 significant digits: w / w+1 agree (final) or the literal is reported unsupported."""
    r = random.Random(9)
    strs = []
    for _ in range(20_000):
        nd = r.randint(20, 40)
        digits = str(r.randint(1, 9)) + "".join(r.choice("0123456789") for _ in range(nd - 1))
        dot = r.randint(1, nd)
        strs.append(digits[:dot] + "." + digits[dot:] + "e" + str(r.randint(-300, 300)))
    n_unsup = check(core, strs, allow_unsupported=True)
    assert n_unsup < 80  # ambiguous only within ~1e-19 relative of a rounding boundary (~1e-3 of them)


def test_halfway_cases_round_to_even(core):
    """Exact midpoints between adjacent doubles: round half to even (short ones must be exact)."""
    strs = ["9007199254740993", "9007199254740995", "4503599627370497.5", "2.5", "0.5e1"]
    r = random.Random(3)
    for _ in range(2000):
        m = r.randint(2**52, 2**53 - 1)
        e = r.randint(-10, 20)
        mid = Fraction(2 * m + 1, 2) * Fraction(2) ** e
        if mid.denominator == 1 and mid.numerator < 10**19:
            strs.append(str(mid.numerator))
    assert check(core, strs) == 0


def test_java_grammar(core):
    good = {"NaN": math.nan, "-NaN": math.nan, "Infinity": math.inf, "-Infinity": -math.inf, "+Infinity": math.inf,
            "  3.25  ": 3.25, "\t-0.0": -0.0, ".5": 0.5, "5.": 5.0, "1.5f": 1.5, "2e3D": 2000.0, "+7": 7.0,
            "1e-400": 0.0, "1e400": math.inf, "4.9e-324": 5e-324, "2.4703282292062328e-324": 5e-324,
            "2.2250738585072011e-308": 2.225073858507201e-308, "1.7976931348623157e308": 1.7976931348623157e308,
            '"116.5"': 116.5, '11"6.25': 116.25, "0000123.4500": 123.45, "0.000000000000000000000012": 1.2e-23}
    for s, e in good.items():
        v = C.c_double()
        assert core.core_parse_double(s.encode(), len(s), C.byref(v)) == OK, s
        assert bits(v.value) == bits(e) or (math.isnan(v.value) and math.isnan(e)), (s, v.value, e)
    for s in ["", " ", ".", "e5", "1e", "1e+", "--1", "1.2.3", "1 5", "NaNx", "Inf", "1.5x", "+", "-.e1", "1ff"]:
        v = C.c_double()
        assert core.core_parse_double(s.encode(), len(s), C.byref(v)) == BAD, s
    v = C.c_double()
    assert core.core_parse_double(b"0x1p3", 5, C.byref(v)) == UNSUP


def test_java_long(core):
    for s, e in {"0": 0, "-12": -12, "+5": 5, "9223372036854775807": 2**63 - 1, "-9223372036854775808": -2**63,
                 '"42"': 42}.items():
        v = C.c_int64()
        assert core.core_parse_long(s.encode(), len(s), C.byref(v)) == OK, s
        assert v.value == e
    for s in ["", "-", "9223372036854775808", "-9223372036854775809", "1.0", " 1", "1 ", "1e3"]:
        v = C.c_int64()
        assert core.core_parse_long(s.encode(), len(s), C.byref(v)) == BAD, s


def test_objid_canonical_keys(core):
    """objID Strings (Deserialization.java:317) take the numeric key only when the String is
    Long.toString(v) of v in [-2^62, 2^62) (quotes are removed before the split): the key map is
    injective over Strings -- "7" and "007" / "+7" / " 7" / "-0" never share a key."""
    core.core_objid_key.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
    rng = random.Random(3)
    cases = ["0", "7", "-7", "-0", "00", "007", "+7", " 7", "7 ", "", "-", "abc", "1e3", "12a",
             str(2**62 - 1), str(2**62), str(-(2**62)), str(-(2**62) - 1), str(2**63 - 1), "9" * 19, "9" * 20,
             '"7"', '7"', '"-"12']
    cases += [str(rng.randint(-2**63, 2**63 - 1)) for _ in range(2000)]
    cases += [str(rng.randint(-10**6, 10**6)) for _ in range(2000)]
    for s in cases:
        v = C.c_int64()
        ok = core.core_objid_key(s.encode(), len(s), C.byref(v))
        t = s.replace('"', "")
        canon = t.lstrip("-").isdigit() and str(int(t)) == t and -(2**62) <= int(t) < 2**62
        assert ok == canon, s
        if ok:
            assert v.value == int(t), s
