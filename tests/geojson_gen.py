"""Generator of GeoJSON point-stream lines for the ingest parity tests: the records the reference
reads (Deserialization.GeoJSONToTSpatial, Deserialization.java:149-211: the Kafka ObjectNode
{"key": .., "value": ..}) -- or, for value_lines, the record values themselves (a Feature as
Serialization.PointToGeoJSONOutputSchema writes it, Serialization.java:17-50) -- with the
variations a JSON producer may emit: member order, whitespace, number spellings, 3-D
coordinates, value-level Point geometries (taken before the "geometry" member,
readGeoJSON(value) first), Features whose own "type" is missing / not a String / unknown or a
Point with unusable coordinates (the catch branch), numeric / textual / missing objIDs, integer or
date-string timestamps (with lenient field rollover), duplicate keys, nested noise with literals.
Every generated line is valid for the map (no error line)."""
import json

import numpy as np


def _num(rng, v):
    k = rng.integers(0, 5)
    if k == 0:
        return repr(float(v))
    if k == 1:
        return f"{v:.6f}"
    if k == 2:
        return f"{v / 100:.9f}E2"
    if k == 3:
        return f"{v:.17g}"
    return str(int(round(v))) if rng.random() < 0.2 else repr(float(v))


def _date(rng):
    if rng.random() < 0.15:  # lenient rollover
        return f"{rng.integers(1990, 2030)}-{rng.integers(1, 15)}-{rng.integers(0, 40)} " \
               f"{rng.integers(0, 30)}:{rng.integers(0, 70)}:{rng.integers(0, 70)}"
    if rng.random() < 0.05:
        return "not a date"
    return f"{rng.integers(1990, 2030)}-{rng.integers(1, 13):02d}-{rng.integers(1, 29):02d} " \
           f"{rng.integers(0, 24):02d}:{rng.integers(0, 60):02d}:{rng.integers(0, 60):02d}"


def _coords(rng, xs, ys):
    if rng.random() < 0.15:
        return f"[{xs},{ys},{rng.integers(-5, 90)}.5]"  # z ordinate
    return f"[{xs}, {ys}]" if rng.random() < 0.5 else f"[{xs},{ys}]"


def _props(rng, date_fmt):
    props = []
    ok = rng.integers(0, 12)
    if ok < 4:
        props.append(f'"oID":"{rng.integers(0, 10**6)}"')
    elif ok < 6:
        props.append(f'"oID":{rng.integers(-10**12, 10**12)}')
    elif ok == 6:
        props.append('"oID":"bus-' + "".join(rng.choice(list("abcxyz09"), int(rng.integers(1, 9)))) + '"')
    elif ok == 7:
        props.append('"oID":"007"')
    elif ok == 8:
        props.append(f'"oID":{rng.choice(["true", "false", "null", "-0", "0"])}')
    elif ok == 9:
        props.append('"oID":"stale","oID":"' + str(rng.integers(0, 99)) + '"')  # the last duplicate wins
    # ok 10, 11: no objID
    tk = rng.integers(0, 10)
    if tk < 8:
        props.append(f'"timestamp":"{_date(rng)}"' if date_fmt else f'"timestamp":{rng.integers(0, 2**41)}')
    if rng.random() < 0.3:
        props.append('"meta":{"s":"}{][,:","a":[1,{"b":[2,3e5,-0.5E-3]}],"n":null,"t":true,"f":false}')
    rng.shuffle(props)
    return "{" + ", ".join(props) + "}"


def _value(rng, xs, ys, date_fmt):
    """A record value the map reads to (xs, ys)."""
    shape = rng.integers(0, 20)
    members = []
    if shape < 3:  # the value is itself a Point geometry (readGeoJSON(value) succeeds)
        members += ['"type":"Point"', f'"coordinates":{_coords(rng, xs, ys)}']
        if rng.random() < 0.3:  # a geometry member too: the value's own point wins
            members.append('"geometry":{"type":"Point","coordinates":[1.5,2.5]}')
    else:
        geom = [f'"coordinates":{_coords(rng, xs, ys)}', '"type":"Point"']
        rng.shuffle(geom)
        members.append(f'"geometry":{{{",".join(geom)}}}')
        if shape < 14:
            members.append('"type":"Feature"')
        elif shape == 14:
            members.append('"type":7')  # not a String: ClassCastException -> the catch branch
        elif shape == 15:
            members.append('"type":"Thing"')  # unknown type -> the catch branch
        elif shape == 16:  # a Point whose coordinates JTS cannot read -> the catch branch
            members += ['"type":"Point"', rng.choice(['"coordinates":"x"', '"coordinates":[true,1]',
                                                      '"coordinates":[[1,2]]', '"coordinates":null'])]
        # shape 17..19: no "type" at all -> the catch branch
    if rng.random() < 0.9:
        members.append(f'"properties":{_props(rng, date_fmt)}')
    rng.shuffle(members)
    return "{" + ",".join(members) + "}"


def lines(seed, n, date_fmt, bounds=(115.5, 117.6, 39.6, 41.1), value_lines=False):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        x = rng.uniform(bounds[0], bounds[1])
        y = rng.uniform(bounds[2], bounds[3])
        v = _value(rng, _num(rng, x), _num(rng, y), date_fmt)
        if value_lines:
            out.append(v)
            continue
        key = rng.choice([str(i), f'"{i}"', "null", f'{{"id":{i}}}'])
        r = rng.random()
        if r < 0.05:  # an earlier "value" member: the last one wins
            out.append(f'{{"value":{{"type":"Point","coordinates":[0,0]}},"key":{key},"value":{v}}}')
        elif r < 0.5:
            out.append(f'{{"key":{key},"value":{v}}}')
        else:
            out.append(f'{{"value":{v}, "key":{key}}}')
    return ("\n".join(out) + "\n").encode()


def check_json(text):
    for ln in text.split(b"\n"):
        if ln:
            json.loads(ln)


# ---- hand-built lines shared by the parity tests (tests/test_gpu_geojson.py, tests/test_geojson_core.py)
G = b'"geometry":{"type":"Point","coordinates":[1,2]}'
BAD = [  # (line, kind): every failure path of the map (the oracle's kinds, tests/test_geojson_oracle.py)
    (b"", 4),
    (b'{"value":{"geometry":{"type":"Point"}}}', 3),
    (b'{"value":{"geometry":{"coordinates":[1,2]}}}', 3),
    (b'{"value":{"geometry":{"type":7,"coordinates":[1,2]}}}', 3),
    (b'{"value":{"geometry":{"type":"Thing","coordinates":[1,2]}}}', 3),
    (b'{"value":{"properties":{}}}', 3),
    (b'{"type":"Feature",' + G + b'}', 3),
    (b'{"value":7}', 3),
    (b'{"value":{"geometry":{"type":"Point","coordinates":["1",2]}}}', 1),
    (b'{"value":{"geometry":{"type":"Point","coordinates":[1]}}}', 2),
    (b'{"value":{"geometry":{"type":"Point","coordinates":[1,2,"z"]}}}', 2),
    (b'{"value":{"geometry":{"type":"LineString","coordinates":[[1,2],[3,4]]}}}', 2),
    (b'{"value":{"type":"Polygon","coordinates":[[[1,2],[3,4],[5,6],[1,2]]]}}', 2),
    (b'{"value":{"type":"FeatureCollection","features":[]}}', 2),
    (b'{"value":{' + G + b',"properties":{"timestamp":1.5}}}', 1),
    (b'{"value":{' + G + b',"properties":{"oID":2.5}}}', 2),
    (b'{"value":{' + G + b',"properties":{"oID":"a\\"b"}}}', 2),
    (b'{"value":{' + G + b',"properties":{"o\\u0049D":"a"}}}', 2),
    (b'{"value":{"geometry":{"type":"Point","coordinates":[1,2]', 3),
    (b'{"value":{' + G + b',"n":NaN}}', 3),
    (b'{"value":{' + G + b',"n":-Infinity}}', 3),
    (b'{"value":{' + G + b',"n":Infinity}}', 3),
    (b'{"value":{' + G + b',"n":nan}}', 3),
    (b'{"value":{' + G + b',"n":tru}}', 3),
    (b'{"value":{' + G + b',"n":01}}', 3),
    (b'{"value":{' + G + b',"n":1.}}', 3),
    (b'{"value":{' + G + b',"n":+1}}', 3),
    (b'{"value":{' + G + b',"n":"a\tb"}}', 3),
    (b'{"value":{' + G + b',"n":"\xe9t\xc3"}}', 3),
    (b'{"value":{' + G + b',"n":"\\q"}}', 3),
    (b'{"value":{' + G + b'}} x', 3),
    (b'{"value":{' + G + b'}},', 3),
    (b'{"value":{' + G + b',"n":1e400}}', 2),
    (b'{"value":{' + G + b',"n":-1.5E+308999}}', 2),
    (b'{"value":{' + G + b',"n":99999999999999999999}}', 2),
    (b'{"value":{' + G + b',"n":' + b"[" * 300 + b"]" * 300 + b'}}', 2),
]



DEEP = b'{"value":{' + G + b',"x":' + b"[" * 70 + b"]" * 70 + b'}}'
V = b'"value":'
TRICKY = [  # valid lines the one-pass locator takes (or hands to the walk: escapes, depth > 63, long numbers)
    b'{"value":{' + G + b'},"value":{"geometry":{"type":"Point","coordinates":[3,4]},"properties":{"oID":"a"}}}',
    b'{"value":{"geometry":{"type":"Point","coordinates":[1,2],"coordinates":[5,6]}}}',
    b'{"value":{"geometry":{"type":"Point","coordinates":[1,2]},"geometry":{"type":"Point","coordinates":[3,4]}}}',
    b'{"value":{"type":"Point","coordinates":[7,8],"geometry":{"type":"Point","coordinates":[3,4]}}}',
    b'{"value":{"coordinates":[7,8],"type":"Point"}}',
    b'{"value":{"type":"Point","coordinates":[[7,8]],"geometry":{"type":"Point","coordinates":[3,4]}}}',
    b'{"value":{"type":"Point","coordinates":{"a":1},"geometry":{"type":"Point","coordinates":[3,4]}}}',
    b'{"value":{"type":"Point","coordinates":null,"geometry":{"type":"Point","coordinates":[3,4]}}}',
    b'{"value":{"type":"Point","coordinates":[true,1],"geometry":{"type":"Point","coordinates":[3,4]}}}',
    b'{"value":{"type":"Poin","geometry":{"type":"Point","coordinates":[3,4]}}}',
    b'{"value":{"type":null,' + G + b'}}',
    b'{"value":{"type":["Point"],' + G + b'}}',
    b'{"a":[{' + V + b'{"type":"Point","coordinates":[9,9]}}],"value":{' + G + b',"properties":{"p":{"oID":3},"oID":"7"}}}',
    b'{"value":{"value":{"type":"Point","coordinates":[0,0]},' + G + b'}}',
    b'{"value":{"properties":{"timestamp":1,"oID":2},' + G + b',"properties":[1,2]}}',
    ' { "value" : { "geometry" : { "type" : "Point" , "coordinates" : [ 1 , 2 ] } , "properties" : { "oID" : "é☃" } } } '.encode(),
    DEEP,
    b'{"value":{' + G + b',"properties":{"coordinates":1,"timestamp":2,"oIDx":3,"oI":4}}}',
    b'{"value":{"geometry":{"type":"Point","coordinates":[1e-3,2E+1,3]},"properties":{}}}',
    b'{"s":"}{][,:",' + V + b'{' + G + b',"properties":{"oID":"q"}}}',
    b'{"s":"a\\"b\\u0041\\n",' + V + b'{' + G + b',"properties":{"oID":"q","timestamp":3}}}',
    b'{"":1,' + V + b'{' + G + b',"properties":{"oID":true,"timestamp":-0}}}',
    b'{"key":{"geometry":{"coordinates":[3,4]}},"value":{' + G + b',"properties":{"oID":6}}}',
    b'{"value":{' + G + b',"properties":{"oID":null,"timestamp":-12}}}',
    b'{"key":1,"value":{"type":"Feature","geometry":{"coordinates":[1e-3,2E+1],"type":"Point"},"properties":{"oID":-5}}}',
    b'{"key":123456789012345678,"value":{' + G + b',"q":1.5e300,"r":12345678901234567890.5,"t":[true,false,null]}}',
    b'{"value":{"geometry":{"type":"Point","coordinates":[-0,-0.0]},"properties":{"oID":"\xc3\xa9\xe2\x98\x83\xf0\x9f\x98\x80"}}}',
    b'{"value":{"type":"Point","coordinates":[1.7976931348623157e308,-4.9e-324]}}',
]


