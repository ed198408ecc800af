"""CPU: the GeoJSON ingest oracle (oracle.geojson_parse, a restatement of
Deserialization.GeoJSONToTSpatial.map, Deserialization.java:149-211, over Python's json module)
pinned to the reference's own documented example (Deserialization.java:120-121: the Kafka
record {"key":136138,"value":{... [116.44412,39.93984] ... "oID":"2560" ...}}) and to the
semantics the map's code spells out, case by case: readGeoJSON(value) first, the catch branch's
value.get("geometry") second (:136-141, :172-178), Jackson's strict reading of the record."""
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


G = b'"geometry":{"type":"Point","coordinates":[1,2]}'


@pytest.mark.parametrize("line,exp", [
    # the value is a bare Point geometry: readGeoJSON(value) succeeds, no properties
    (b'{"key":1,"value":{"type":"Point","coordinates":[5,6]}}', (5.0, 6.0, None, 0)),
    # ... and its own point wins over a "geometry" member; properties are the value's
    (b'{"value":{"type":"Point","coordinates":[5,6,7],' + G + b',"properties":{"oID":7,"timestamp":5}}}',
     (5.0, 6.0, b"7", 5)),
    # a Point with unreadable coordinates, a Feature, no type, a non-string or unknown type: the catch branch
    (b'{"value":{"type":"Point","coordinates":[[5,6]],' + G + b'}}', (1.0, 2.0, None, 0)),
    (b'{"value":{"type":"Point","coordinates":"x",' + G + b'}}', (1.0, 2.0, None, 0)),
    (b'{"value":{"type":"Feature",' + G + b'}}', (1.0, 2.0, None, 0)),
    (b'{"value":{' + G + b'}}', (1.0, 2.0, None, 0)),
    (b'{"value":{"type":5,' + G + b'}}', (1.0, 2.0, None, 0)),
    (b'{"value":{"type":"Thing",' + G + b'}}', (1.0, 2.0, None, 0)),
    # an integer literal is (double) of Jackson's IntNode: "-0" -> +0.0; "-0" objID prints as 0;
    # duplicate keys: the last wins
    (b'{"value":{"type":"Point","coordinates":[-0,-0.0],"properties":{"oID":-0,"timestamp":1,"timestamp":9}}}',
     (0.0, -0.0, b"0", 9)),
    (b'{"value":{' + G + b',"properties":{"oID":null}}}', (1.0, 2.0, b"null", 0)),
    (b'{"value":{' + G + b',"properties":{"oID":true}}}', (1.0, 2.0, b"true", 0)),
    (b'{"value":{' + G + b',"properties":null}}', (1.0, 2.0, None, 0)),
    # the last "value" member is the record's value
    (b'{"value":{"type":"Point","coordinates":[8,9]},"value":{' + G + b'}}', (1.0, 2.0, None, 0)),
    # a big integer / float elsewhere that json-simple reads back is fine
    (b'{"key":123456789012345678,"value":{' + G + b',"q":1.5e300}}', (1.0, 2.0, None, 0)),
])
def test_cases(oracle_mod, line, exp):
    import math

    x, y, o, t, bl, bk = oracle_mod.geojson_parse(line, "oID", "timestamp", 0, 0)
    assert bl == -1, bk
    assert (x[0], y[0], o[0], t[0]) == exp
    assert math.copysign(1, x[0]) == math.copysign(1, exp[0]) and math.copysign(1, y[0]) == math.copysign(1, exp[1])


def test_value_lines(oracle_mod):
    feat = b'{"type":"Feature",' + G + b',"properties":{"oID":"a"}}'
    x, y, o, t, bl, bk = oracle_mod.geojson_parse(feat, "oID", None, 0, 0, value_lines=True)
    assert bl == -1 and (x[0], y[0], o[0]) == (1.0, 2.0, b"a")
    *_, bl, bk = oracle_mod.geojson_parse(feat, "oID", None, 0, 0)  # a record without "value": NPE
    assert (bl, bk) == (0, 3)


@pytest.mark.parametrize("line,kind", [
    (b"", 4),
    (b'{"value":{"geometry":{"type":"Point"}}}', 3),                        # no coordinates
    (b'{"value":{"geometry":{"coordinates":[1,2]}}}', 3),                   # geometry without a type
    (b'{"value":{"geometry":{"type":7,"coordinates":[1,2]}}}', 3),          # non-string type
    (b'{"value":{"geometry":{"type":"Thing","coordinates":[1,2]}}}', 3),    # unknown type
    (b'{"value":{"properties":{}}}', 3),                                     # no geometry
    (b'{"type":"Feature",' + G + b'}', 3),                                   # no "value": NPE
    (b'{"value":7}', 3),
    (b'{"value":{"geometry":{"type":"Point","coordinates":["1",2]}}}', 1),  # not a number
    (b'{"value":{"geometry":{"type":"Point","coordinates":[1]}}}', 2),      # JTS's default ordinate
    (b'{"value":{"geometry":{"type":"Point","coordinates":[1,2,"z"]}}}', 2),
    (b'{"value":{"geometry":{"type":"LineString","coordinates":[[1,2],[3,4]]}}}', 2),
    (b'{"value":{"type":"Polygon","coordinates":[[[1,2],[3,4],[5,6],[1,2]]]}}', 2),
    (b'{"value":{"type":"FeatureCollection","features":[]}}', 2),
    (b'{"value":{' + G + b',"properties":{"timestamp":1.5}}}', 1),          # parseLong("1.5")
    (b'{"value":{' + G + b',"properties":{"timestamp":"12"}}}', 1),         # parseLong("\"12\"")
    (b'{"value":{' + G + b',"properties":{"oID":2.5}}}', 2),                # Double.toString: not restated
    (b'{"value":{' + G + b',"properties":{"oID":"a\\"b"}}}', 2),            # escaped string
    (b'{"value":{' + G + b',"properties":{"o\\u0049D":"a"}}}', 2),          # escaped member name
    (b'{"value":{"geometry":{"type":"Point","coordinates":[1,2]', 3),       # malformed JSON
    (b'{"value":{' + G + b',"n":NaN}}', 3),                                 # Jackson refuses NaN
    (b'{"value":{' + G + b',"n":-Infinity}}', 3),
    (b'{"value":{' + G + b',"n":tru}}', 3),
    (b'{"value":{' + G + b',"n":01}}', 3),
    (b'{"value":{' + G + b',"n":"a\tb"}}', 3),                              # unescaped control byte
    (b'{"value":{' + G + b',"n":"\xe9t\xc3"}}', 3),                         # broken UTF-8
    (b'{"value":{' + G + b'}} x', 3),                                       # content after the record
    (b'{"value":{' + G + b',"n":1e400}}', 2),                               # json-simple cannot read Infinity
    (b'{"value":{' + G + b',"n":99999999999999999999}}', 2),                # ... nor an integer outside long
    (b'{"value":{' + G + b',"n":' + b"[" * 300 + b"]" * 300 + b'}}', 2),    # nesting > 256
])
def test_errors(oracle_mod, line, kind):
    *_, bl, bk = oracle_mod.geojson_parse(line, "oID", "timestamp", 0, 0)
    assert (bl, bk) == (0, kind)


def test_dates(oracle_mod):
    import calendar

    def ms(s, tz=0):
        ln = b'{"value":{' + G + b',"properties":{"t":"' + s.encode() + b'"}}}'
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


def test_generator_is_valid_json_and_error_free(oracle_mod):
    for fmt in (0, 1):
        for vl in (False, True):
            text = lines(5, 2000, fmt, value_lines=vl)
            check_json(text)
            *_, bl, bk = oracle_mod.geojson_parse(text, "oID", "timestamp", fmt, 0, value_lines=vl)
            assert bl == -1, (fmt, vl, bk, text.split(b"\n")[bl])
