"""GPU: GeoJSON point ingest (gf_geojson_parse, the device restatement of
Deserialization.GeoJSONToTSpatial.map, Deserialization.java:149-211) against the oracle
(oracle.geojson_parse, over Python's json module): x / y bit-exact, ts, objID Strings (decoded
from the keys; None for a null objID), cells, and the first bad line with its kind."""
import ctypes
import numpy as np
import pytest

from conftest import BEIJING
from geojson_gen import BAD, G, TRICKY, lines

C_ULL4 = ctypes.c_ulonglong * 4

pytestmark = pytest.mark.gpu

REF = (b'{"key":136138,"value":{"geometry":{"coordinates":[116.44412,39.93984],"type":"Point"},'
       b'"properties":{"oID":"2560","timestamp":"2008-02-02 20:12:32"},"type":"Feature"}}')


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def parse(sf, text, date_fmt=None, tz=0, grid=None, props=("oID", "timestamp"), value_lines=False):
    d = sf.Deserialization.GeoJSONToTSpatial(grid, date_fmt, props[1], props[0], tz_offset_minutes=tz,
                                             value_lines=value_lines)
    return d.parse(text)


def check(sf, oracle_mod, text, date_fmt, tz, grid=None, og=None, value_lines=False):
    w = parse(sf, text, date_fmt, tz, grid, value_lines=value_lines)
    ex, ey, eo, et, bl, bk = oracle_mod.geojson_parse(text, "oID", "timestamp", 1 if date_fmt else 0, tz, value_lines)
    assert bl == -1
    np.testing.assert_array_equal(w.x.cpu().numpy().view(np.uint64), ex.view(np.uint64))
    np.testing.assert_array_equal(w.y.cpu().numpy().view(np.uint64), ey.view(np.uint64))
    np.testing.assert_array_equal(w.timeStampMillisec.cpu().numpy(), et)
    got = w.objid_strings()
    assert got == [None if o is None else o.decode() for o in eo]
    if grid is not None:
        cx, cy = oracle_mod.assign_cells(og, ex, ey)
        np.testing.assert_array_equal(w.extra["cx"].cpu().numpy(), cx)
        np.testing.assert_array_equal(w.extra["cy"].cpu().numpy(), cy)
    return w


def test_reference_example(sf, oracle_mod):
    w = check(sf, oracle_mod, REF + b"\n", "yyyy-MM-dd HH:mm:ss", 480)
    assert w.objid_strings() == ["2560"] and int(w.objID[0]) == 2560  # canonical decimal: its value
    assert int(w.timeStampMillisec[0]) == 1201954352000


@pytest.mark.parametrize("seed,n,date_fmt,tz,vl", [(1, 50_000, None, 0, False),
                                                   (2, 50_000, "yyyy-MM-dd HH:mm:ss", 480, False),
                                                   (3, 3_000, "yyyy-MM-dd HH:mm:ss", -300, False), (4, 1, None, 0, False),
                                                   (5, 40_000, None, 0, True), (6, 3_000, "yyyy-MM-dd HH:mm:ss", 60, True)])
def test_generated_lines(sf, oracle_mod, seed, n, date_fmt, tz, vl):
    g = sf.UniformGrid(100, *BEIJING)
    check(sf, oracle_mod, lines(seed, n, 1 if date_fmt else 0, value_lines=vl), date_fmt, tz, g,
          oracle_mod.grid(100, *BEIJING), value_lines=vl)


def test_crlf_and_missing_final_newline(sf, oracle_mod):
    text = lines(9, 200, 0).replace(b"\n", b"\r\n").rstrip(b"\r\n")
    check(sf, oracle_mod, text, None, 0)


def test_no_property_names(sf):
    w = parse(sf, REF + b"\n", None, 0, None, (None, None))  # objID always null, time 0
    assert w.objid_strings() == [None] and int(w.timeStampMillisec[0]) == 0


@pytest.mark.parametrize("walk", [0, 1])
def test_first_bad_line(sf, oracle_mod, walk):
    """Each bad line inside a chunk of good ones: the chunk fails at that line with the oracle's kind
    (the locator's strict check sends every one of them to the walk, which decides)."""
    from spatialflink_amd import _lib
    good = lines(11, 300, 0).split(b"\n")[:300]
    ctx = _lib.context(0)
    _lib.check(_lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_GEOJSON_WALK, walk), ctx.handle, "flag")
    try:
        for bad, kind in BAD:
            text = b"\n".join(good[:137] + [bad] + good[137:]) + b"\n"
            *_, bl, bk = oracle_mod.geojson_parse(text, "oID", "timestamp", 0, 0)
            assert (bl, bk) == (137, kind), bad
            with pytest.raises(ValueError, match=f"line 137: {sf.spatialStreams.CSV_KINDS[kind]}"):
                parse(sf, text)
    finally:
        _lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_GEOJSON_WALK, 0)


@pytest.mark.parametrize("walk", [0, 1])
def test_locator_matches_walk(sf, oracle_mod, walk):
    """The one-pass member locator (k_csv.hip geo_locate) and the member-by-member walk it stands
    in for give the oracle's results on generated lines plus valid records built to exercise
    last-wins duplicates at each level, the value's own Point before its geometry, every catch-
    branch trigger, members inside arrays and deeper objects, whitespace, UTF-8 (2-4 byte
    sequences), structural bytes inside strings, escapes in members not taken, literals, long and
    3-digit-exponent numbers json-simple reads back, -0 ordinates and nesting deeper than the
    locator's stack.  (Malformed / unsupported lines: test_first_bad_line, both paths.)"""
    from spatialflink_amd import _lib
    text = lines(21, 5_000, 0) + b"\n".join(TRICKY * 40) + b"\n"
    ctx = _lib.context(0)
    _lib.check(_lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_GEOJSON_WALK, walk), ctx.handle, "flag")
    try:
        check(sf, oracle_mod, text, None, 0)
    finally:
        _lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_GEOJSON_WALK, 0)


NUMS = [b"0", b"-0", b"00", b"01", b"-01", b"0.", b".5", b"1.", b"1.5", b"1.5.3", b"1e", b"1e+", b"1e5", b"1E-5",
        b"1e05", b"1e123", b"1e12", b"-1.25e+07", b"1e5e3", b"1.5e3.2", b"--1", b"1-2", b"+1", b"-", b"1+2",
        b"123456789012345678", b"1234567890123456789", b"-12345678901234567", b"-123456789012345678",
        b"0.000000000000001", b"0.0000000000000001", b"1.5E", b"2e-", b"true", b"tru", b"truex", b"false",
        b"null", b"nul", b"nulll", b"t", b"e5", b"E", b"1x", b"0x10", b"Infinity", b"NaN", b"1.0e-2"]


def _fuzz_lines(seed, n):
    """Generated lines with 1-3 random ASCII edits (deletions, structural / token bytes inserted,
    swaps, duplicated spans): a mix of valid and malformed records for the acceptance check."""
    rng = np.random.default_rng(seed)
    base = lines(seed, n, 0).split(b"\n")[:n]
    alphabet = b'{}[]:,"0123456789.eE+-tfnul \t'
    out = []
    for ln in base:
        b = bytearray(ln)
        for _ in range(int(rng.integers(1, 4))):
            k = int(rng.integers(0, 4))
            pos = int(rng.integers(1, max(2, len(b))))
            if k == 0 and len(b) > 2:
                del b[pos % len(b)]
            elif k == 1:
                b.insert(pos, alphabet[int(rng.integers(0, len(alphabet)))])
            elif k == 2 and len(b) > 3:
                q = int(rng.integers(1, len(b)))
                b[pos % len(b)], b[q] = b[q], b[pos % len(b)]
            else:
                q = min(len(b), pos + int(rng.integers(1, 12)))
                b[pos:pos] = b[pos:q]
        out.append(bytes(b).replace(b"\n", b" "))
    return out


def _shifted(lines_, width=64):
    """Each line with 0..width-1 blanks after its '{': every byte at every step offset of the scan."""
    out = []
    for ln in lines_:
        i = ln.find(b"{")
        for k in range(width):
            out.append(ln[:i + 1] + b" " * k + ln[i + 1:])
    return out


@pytest.mark.parametrize("vl", [False, True])
def test_wave_scan_matches_lane_locator(sf, oracle_mod, vl):
    """The wave-per-line scan (k_csv.hip geo_wave_scan) against the lane locator it replaces, on
    every staged line (GF_FLAG_GEOJSON_CHECK): it never passes a line the locator sends to the
    walk and its member notes are the locator's; on ASCII lines it passes every line the locator
    passes.  Corpora: generated lines, the tricky and bad lines, numbers and literals of every
    grammar edge, each shifted across the 64-byte step boundaries, and random edits."""
    from spatialflink_amd import _lib
    L = _lib.lib()
    ctx = _lib.context(0)
    num_lines = [b'{"value":{' + G + b',"n":' + v + b',"m":[' + v + b"," + v + b']}}' for v in NUMS]
    keys = [b'{"value":{"geometry":{"type":"Point","coordinates":[1,2]},"properties":{"' + b"x" * k +
            b'":1,"oID":"' + b"y" * k + b'","timestamp":' + b"7" * min(k + 1, 18) + b"}}}" for k in range(0, 70, 3)]
    if vl:
        corpora = [lines(61, 3000, 0, value_lines=True).split(b"\n")[:3000],
                   _shifted([ln[ln.find(b":{") + 1:-1] for ln in num_lines[:12] + keys[:6]])]
    else:
        ascii_ = [t for t in TRICKY if max(t) < 0x80]
        corpora = [lines(62, 4000, 0).split(b"\n")[:4000], _shifted(ascii_, 64), _shifted(num_lines, 64),
                   _shifted(keys), _shifted([b for b, _ in BAD if b and max(b) < 0x80], 24), _fuzz_lines(63, 6000)]
    _lib.check(L.gf_ctx_set_flag(ctx.handle, _lib.FLAG_GEOJSON_CHECK, 1), ctx.handle, "flag")
    try:
        for ci, corpus in enumerate(corpora):
            text = b"\n".join(corpus) + b"\n"
            assert max(text) < 0x80
            cnt = (C_ULL4)()
            for _ in range(2):  # (the first call sizes the LDS staging from its mean line: the second stages all)
                try:
                    parse(sf, text, value_lines=vl)
                except ValueError:
                    pass  # malformed lines: the check counts every line all the same
                _lib.check(L.gf_geojson_check_counts(ctx.handle, cnt), ctx.handle, "counts")
            both, scan_only, differ, lane_only = list(cnt)
            assert scan_only == 0 and differ == 0, (ci, list(cnt))
            assert lane_only == 0, (ci, list(cnt))
            assert both > 0, (ci, list(cnt))
    finally:
        L.gf_ctx_set_flag(ctx.handle, _lib.FLAG_GEOJSON_CHECK, 0)


@pytest.mark.parametrize("wave", [0, 1])
def test_generated_lines_wave_and_lane(sf, oracle_mod, wave):
    """The lane locator (default) and the wave scan give the oracle's results on the same lines."""
    from spatialflink_amd import _lib
    ctx = _lib.context(0)
    _lib.check(_lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_GEOJSON_WAVE, wave), ctx.handle, "flag")
    try:
        text = lines(71, 20_000, 0) + b"\n".join(_shifted(TRICKY[:20], 64)) + b"\n"
        check(sf, oracle_mod, text, None, 0)
    finally:
        _lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_GEOJSON_WAVE, 0)
