"""Generator of GeoJSON point-stream lines for the ingest parity tests: the shapes the reference
reads (Deserialization.GeoJSONToTSpatial, Deserialization.java:149-211) and writes
(Serialization.PointToGeoJSONOutputSchema, Serialization.java:17-50) -- Kafka key/value records
and bare Features -- with the variations a JSON producer may emit: member order, whitespace,
number spellings, nested coordinate arrays, numeric / textual / missing objIDs, integer or
date-string timestamps (with lenient field rollover), duplicate keys, nested noise."""
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


def lines(seed, n, date_fmt, bounds=(115.5, 117.6, 39.6, 41.1)):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        x = rng.uniform(bounds[0], bounds[1])
        y = rng.uniform(bounds[2], bounds[3])
        gk = rng.integers(0, 10)
        xs, ys = _num(rng, x), _num(rng, y)
        if gk < 7:
            coords = f"[{xs}, {ys}]" if rng.random() < 0.5 else f"[{xs},{ys}" + (",12.5]" if rng.random() < 0.2 else "]")
            gtype = "Point"
        elif gk < 9:
            coords = f"[[{xs},{ys}],[116.1,40.2]]"
            gtype = "LineString"
        else:
            coords = f"[[[{xs},{ys}],[116.1,40.2],[116.2,40.3],[{xs},{ys}]]]"
            gtype = "Polygon"
        geom = [f'"coordinates":{coords}', f'"type":"{gtype}"']
        rng.shuffle(geom)
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
            props.append('"meta":{"s":"}{][,:","a":[1,{"b":[2,3]}],"n":null}')
        rng.shuffle(props)
        feat = [f'"geometry":{{{",".join(geom)}}}', '"type":"Feature"']
        if rng.random() < 0.9:
            feat.append(f'"properties":{{{", ".join(props)}}}')
        rng.shuffle(feat)
        f = "{" + ",".join(feat) + "}"
        out.append(f'{{"key":{i},"value":{f}}}' if rng.random() < 0.6 else f)
    return ("\n".join(out) + "\n").encode()


def check_json(text):
    for ln in text.split(b"\n"):
        if ln:
            json.loads(ln)
