"""CPU: the GeoJSON ingest oracle (oracle.geojson_parse, a restatement of
Deserialization.GeoJSONToTSpatial.map, Deserialization.java:149-211, over Python's json module)
pinned to the reference's own documented example (Deserialization.java:120-121: the Kafka
record {"key":136138,"value":{... [116.44412,39.93984] ... "oID":"2560" ...}}) and to the
semantics the map's code spells out, case by case."""
import numpy as np
import pytest

from geojson_gen import check_json, lines

REF = (b'{"key":136138,"value":{"geometry":{"coordinates":[116.44412,39.93984],"type":"Point"},'
       b'"properties":{"oID":"2560","timestamp":"2008-02-02 20:12:32"},"type":"Feature"}}')


def test_reference_example(oracle_mod):
    x, y, o, t, bl, bk = oracle_mod.geojson_parse(REF + b"\n", "oID", "timestamp", 1, 8 * 60)
    assert bl == -1 and x[0] == 116.44412 and y[0] == 39.93984 and o == [b"2560"]
    assert t[0] == 1201954352000  # 2008-02-02 20:12:32 at UTC+8 = 12:12:32 UTC
    # dateFormat null: Long.parseLong("\"2008-...\"") throws
    *_, bl, bk = oracle_mod.geojson_parse(REF, "oID", "timestamp", 0, 0)
    assert (bl, bk) == (0, 1)


@pytest.mark.parametrize("line,exp", [
    # bare Feature (Serialization's output), integer ms, numeric objID
    (b'{"type":"Feature","geometry":{"type":"Point","coordinates":[1,2]},"properties":{"oID":7,"timestamp":5}}',
     (1.0, 2.0, b"7", 5)),
    # no properties: objID null, time 0
    (b'{"geometry":{"coordinates":[1.5,2.5]}}', (1.5, 2.5, None, 0)),
    # first coordinate of a polygon; "-0" prints as 0; duplicate key: the last wins
    (b'{"geometry":{"coordinates":[[[3,4],[5,6]]]},"properties":{"oID":-0,"oID":-0,"timestamp":1,"timestamp":9}}',
     (3.0, 4.0, b"0", 9)),
    (b'{"geometry":{"coordinates":[1,2]},"properties":{"oID":null}}', (1.0, 2.0, b"null", 0)),
    (b'{"geometry":{"coordinates":[1,2]},"properties":{"oID":true}}', (1.0, 2.0, b"true", 0)),
    (b'{"geometry":{"coordinates":[1,2]},"properties":null}', (1.0, 2.0, None, 0)),
])
def test_cases(oracle_mod, line, exp):
    x, y, o, t, bl, bk = oracle_mod.geojson_parse(line, "oID", "timestamp", 0, 0)
    assert bl == -1
    assert (x[0], y[0], o[0], t[0]) == exp


@pytest.mark.parametrize("line,kind", [
    (b"", 4),
    (b'{"geometry":{"type":"Point"}}', 3),                                        # no coordinates
    (b'{"value":{"properties":{}}}', 3),                                          # no geometry
    (b'{"geometry":{"coordinates":["1",2]}}', 1),                                 # not a number
    (b'{"geometry":{"coordinates":[1]}}', 3),
    (b'{"geometry":{"coordinates":[1,2]},"properties":{"timestamp":1.5}}', 1),    # parseLong("1.5")
    (b'{"geometry":{"coordinates":[1,2]},"properties":{"timestamp":"12"}}', 1),   # parseLong("\"12\"")
    (b'{"geometry":{"coordinates":[1,2]},"properties":{"oID":2.5}}', 2),          # Double.toString: not restated
    (b'{"geometry":{"coordinates":[1,2]},"properties":{"oID":"a\\"b"}}', 2),      # escaped string
    (b'{"geometry":{"coordinates":[1,2]', 3),                                     # malformed JSON
])
def test_errors(oracle_mod, line, kind):
    *_, bl, bk = oracle_mod.geojson_parse(line, "oID", "timestamp", 0, 0)
    assert (bl, bk) == (0, kind)


def test_dates(oracle_mod):
    import calendar

    def ms(s, tz=0):
        ln = b'{"geometry":{"coordinates":[1,2]},"properties":{"t":"' + s.encode() + b'"}}'
        *_, t, bl, bk = oracle_mod.geojson_parse(ln, None, "t", 1, tz)
        return (t[0] if bl < 0 else None), bk

    assert ms("1970-01-01 00:00:00") == (0, 0)
    assert ms("1970-01-01 00:00:00", 60) == (-3600000, 0)
    assert ms("2008-13-01 00:00:00")[0] == calendar.timegm((2009, 1, 1, 0, 0, 0)) * 1000   # month rollover
    assert ms("2008-03-00 24:00:00")[0] == calendar.timegm((2008, 3, 1, 0, 0, 0)) * 1000   # day 0, hour 24
    assert ms("2008-3-2 1:2:3")[0] == calendar.timegm((2008, 3, 2, 1, 2, 3)) * 1000        # short fields
    assert ms("2008-03-02 01:02:03 trailing")[0] == calendar.timegm((2008, 3, 2, 1, 2, 3)) * 1000
    assert ms("2008-03-02")[0] == 0                                                         # ParseException -> 0
    assert ms("1500-01-01 00:00:00") == (None, 2)                                           # Julian calendar


def test_generator_is_valid_json():
    for fmt in (0, 1):
        check_json(lines(5, 2000, fmt))
