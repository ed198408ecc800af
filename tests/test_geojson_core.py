"""CPU: the GeoJSON ingest's per-line evaluator (spatialflink_amd/csrc/gf_geojson.hpp -- the same
code the GPU parse kernel runs per lane, built here for the host by tests/native/geojson_core.cpp)
against the oracle (oracle.geojson_parse over Python's json module), through BOTH of its paths:
the one-pass locator (LDS-staged bytes) and the walk.  x / y bit-exact, ts, objID (canonical key
or the String bytes the dictionary receives) and the kind of every bad line
(Deserialization.GeoJSONToTSpatial.map, Deserialization.java:149-211)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import NATIVE_FLAGS, ROOT
from geojson_gen import BAD, TRICKY, lines

OBJID_NULL = (1 << 63) - 1


@pytest.fixture(scope="module")
def core(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("gcore") / "geojson_core.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", *NATIVE_FLAGS,
                    os.path.join(ROOT, "tests", "native", "geojson_core.cpp"), "-o", out], check=True)
    L = C.CDLL(out)
    L.geojson_core_parse.argtypes = [C.c_char_p, C.c_void_p, C.c_int64, C.c_char_p, C.c_char_p, C.c_int, C.c_int,
                                     C.c_int, C.c_int] + [C.c_void_p] * 8
    return L


def run(core, lns, prop_obj, prop_ts, date_fmt, tz, vl, walk):
    off = np.zeros(len(lns) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in lns])
    buf = b"".join(lns) + b"\0" * 16  # the locator reads whole words past a line's end
    n = len(lns)
    kind = np.zeros(n, np.int32); x = np.zeros(n); y = np.zeros(n); ts = np.zeros(n, np.int64)
    obj = np.zeros(n, np.int64); dic = np.zeros(n, np.int32); ob = np.zeros(n, np.int64); oe = np.zeros(n, np.int64)
    core.geojson_core_parse(buf, off.ctypes.data, n, prop_obj and prop_obj.encode(), prop_ts and prop_ts.encode(),
                            date_fmt, tz, int(vl), int(walk), *(a.ctypes.data for a in (kind, x, y, ts, obj, dic, ob, oe)))
    objs = []
    for i in range(n):
        if dic[i]:
            objs.append(buf[ob[i]:oe[i]])
        elif obj[i] == OBJID_NULL:
            objs.append(None)
        else:
            objs.append(str(int(obj[i])).encode())
    return kind, x, y, ts, objs


def compare(core, oracle_mod, lns, date_fmt=0, tz=0, vl=False, props=("oID", "timestamp")):
    for walk in (0, 1):
        kind, x, y, ts, objs = run(core, lns, props[0], props[1], date_fmt, tz, vl, walk)
        for i, ln in enumerate(lns):
            ex, ey, eo, et, bl, bk = oracle_mod.geojson_parse(ln, props[0], props[1], date_fmt, tz, vl)
            assert kind[i] == (bk if bl == 0 else 0), (walk, ln[:200], kind[i], bk)
            if bl < 0:
                assert x[i].tobytes() == ex[0].tobytes() and y[i].tobytes() == ey[0].tobytes(), (walk, ln[:200])
                assert ts[i] == et[0] and objs[i] == eo[0], (walk, ln[:200], ts[i], et[0], objs[i], eo[0])


@pytest.mark.parametrize("date_fmt,tz,vl", [(0, 0, False), (1, 480, False), (0, 0, True), (1, -300, True)])
def test_generated(core, oracle_mod, date_fmt, tz, vl):
    lns = lines(31 + date_fmt + 2 * vl, 3000, date_fmt, value_lines=vl).split(b"\n")[:-1]
    compare(core, oracle_mod, lns, date_fmt, tz, vl)


def test_tricky_and_bad(core, oracle_mod):
    compare(core, oracle_mod, TRICKY + [b for b, _ in BAD])
    kind, *_ = run(core, [b for b, _ in BAD], "oID", "timestamp", 0, 0, False, 0)
    assert kind.tolist() == [k for _, k in BAD]


def test_no_property_names(core, oracle_mod):
    compare(core, oracle_mod, lines(7, 300, 0).split(b"\n")[:-1] + TRICKY, props=(None, None))


def test_mutations(core, oracle_mod):
    """Every line of a sample with one byte replaced, deleted or duplicated (mostly malformed, some
    still valid): the locator, the walk and the oracle agree on each kind and value."""
    rng = np.random.default_rng(3)
    base = lines(41, 60, 0).split(b"\n")[:-1] + TRICKY[:12]
    alphabet = b'{}[]",:\\ 0123456789.-+eEtfnulrsaI\t\x01\xc3\xa9\x80'
    out = []
    for ln in base:
        for _ in range(12):
            i = int(rng.integers(0, len(ln)))
            op = rng.integers(0, 3)
            c = bytes([alphabet[int(rng.integers(0, len(alphabet)))]])
            out.append(ln[:i] + c + ln[i + 1:] if op == 0 else ln[:i] + ln[i + 1:] if op == 1 else ln[:i] + c + ln[i:])
    compare(core, oracle_mod, out)


@pytest.mark.parametrize("obj_name,ts_name", [("objid_17_chars_xy", "timestamp_abcdef"),   # 17 and 16 bytes
                                              ("a_very_long_object_identifier", "t"),       # 29 and 1
                                              ("oID", "the_time_property_name_longer")])    # 3 and 29
def test_property_name_lengths(core, oracle_mod, obj_name, ts_name):
    """The locator matches member names by (length, 16-byte packed accumulator) and compares names
    longer than 16 bytes byte by byte: property names of 1, 3, 16, 17 and 29 bytes, with decoy
    members whose names share the length (and the last 16 bytes) but not the bytes."""
    lns = lines(53, 400, 0).split(b"\n")[:-1]
    o, t = obj_name.encode(), ts_name.encode()
    decoy_o = (b"X" + o[1:]) if len(o) > 1 else b"Y"
    decoy_t = (b"Z" + t[1:]) if len(t) > 1 else b"W"
    out = []
    for k, ln in enumerate(lns):
        ln = ln.replace(b'"oID"', b'"' + o + b'"').replace(b'"timestamp"', b'"' + t + b'"')
        if k % 3 == 0:  # decoys (same lengths, different first byte) before the real members
            ln = ln.replace(b'"properties": {', b'"properties": {"' + decoy_o + b'": "decoy", "' + decoy_t + b'": 7, ', 1)
            ln = ln.replace(b'"properties":{', b'"properties":{"' + decoy_o + b'":"decoy","' + decoy_t + b'":7,', 1)
        out.append(ln)
    compare(core, oracle_mod, out, props=(obj_name, ts_name))


def test_wave_scan_byte_classes(core):
    """The wave-per-line scan's per-byte table (gf_geojson.hpp wave_class; k_csv.hip geo_wave_scan)
    restated from the JSON lexical rules: every byte in exactly one class, the element it starts
    outside strings, and the number-token sub-flags."""
    import ctypes as C
    out = (C.c_uint32 * 256)()
    core.geojson_core_wave_classes(out)
    WB = dict(Q=1, BAD=2, WSC=4, OTH=8, OB=16, CB=32, OA=64, CA=128, CO=256, CM=512, TOK=1024, DOT=2048, E=4096)
    WT = dict(NONE=0, OB=1, OA=2, CB=3, CA=4, CO=5, CM=6, SK=7, SV=8, TK=9)
    tok = set(b"0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ+-.")
    single = {ord("{"): ("OB", "OB"), ord("}"): ("CB", "CB"), ord("["): ("OA", "OA"), ord("]"): ("CA", "CA"),
              ord(":"): ("CO", "CO"), ord(","): ("CM", "CM"), ord('"'): ("Q", "SV")}
    for b in range(256):
        f, t = out[b] & 0xFFFFFF, out[b] >> 24
        if b in single:
            exp_f, exp_t = WB[single[b][0]], WT[single[b][1]]
        elif b == ord(" "):
            exp_f, exp_t = 0, 0
        elif b in (9, 10, 13):
            exp_f, exp_t = WB["WSC"], 0
        elif b == ord("\\") or b < 0x20 or b >= 0x80:
            exp_f, exp_t = WB["BAD"], 0
        elif b in tok:
            exp_f = WB["TOK"] | (WB["DOT"] if b == ord(".") else 0) | (WB["E"] if b in b"eE" else 0)
            exp_t = WT["TK"]
        else:
            exp_f, exp_t = WB["OTH"], 0
        assert (f, t) == (exp_f, exp_t), (b, f, t, exp_f, exp_t)
