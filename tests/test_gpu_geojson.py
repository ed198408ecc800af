"""GPU: GeoJSON point ingest (gf_geojson_parse, the device restatement of
Deserialization.GeoJSONToTSpatial.map, Deserialization.java:149-211) against the oracle
(oracle.geojson_parse, over Python's json module): x / y bit-exact, ts, objID Strings (decoded
from the keys; None for a null objID), cells, and the first bad line with its kind."""
import numpy as np
import pytest

from conftest import BEIJING
from geojson_gen import BAD, TRICKY, lines

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
