"""GPU parity of the reference's own in-repo callers of the hot path (SURVEY.md §8b "What calls
it"), each at the shape its code spells out, against the oracle:

* Q1_HighRisk (sncb/queries/Q1_HighRisk.java:36,73-78): PointPolygonRangeQuery, RealTime, the
  world grid UniformGrid(100, -180, 180, -90, 90), r = 0.001, the polygon of the reference's
  resource high_risk_zones.geojson (fixture: tests/golden/high_risk_zones_rings.json, made by
  tests/golden/make_callers.py).  The caller first projects the polygon to EPSG:25831 and buffers
  it by 20 m (PolygonLoader.loadGeoJsonResourceBuffered, GeoTools CRS) -- a projection library
  absent here, so the resource polygon is used as read (WGS84 degrees, which is also what the
  degree grid expects).
* MN_Q1 (sncb/mobility/MN_Q1.java:42-66): PointPointRangeQuery, RealTime, the same world grid,
  one query point, the caller's tolMeters handed over as the radius in degrees: 100.0
  (MobilityQueryRunner.java:116-120, Brussels 4.35, 50.85: g = 18 guaranteed and c = 28
  candidate layers -- most of the world grid) and 2.0 (MobilityRunner.java:32, 4.3658, 50.6456:
  g = -1, c = 1).  Points carry String deviceIds (GpsEvent.deviceId -> Point.objID), interned by
  gf_objid_intern, and the emitted points' Strings are decoded back.  The windowAll count per
  5 s tumbling event-time window (MN_Q1.java:68-79) is checked from the hits.

RealTime and WindowBased evaluate the same per-point predicate (the RealTime flatMap bodies equal
the window apply bodies); a RealTime stream is evaluated here batch by batch."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

WORLD = (-180.0, 180.0, -90.0, 90.0)


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def high_risk_rings():
    with open(os.path.join(GOLDEN, "high_risk_zones_rings.json")) as f:
        return json.load(f)["polygons"]


def realtime(sf, approximate=False):
    c = sf.QueryConfiguration(sf.QueryType.RealTime)
    c.setApproximateQuery(approximate)
    return c


def gps_points(seed, n, near, spread):
    """GpsEvent-like stream: most points around `near` (Brussels), some worldwide, plus the
    LocalTestRunner.sampleData() positions (LocalTestRunner.java:86-115); String deviceIds."""
    rng = np.random.default_rng(seed)
    m = n * 3 // 4
    x = np.concatenate([near[0] + rng.uniform(-spread, spread, m), rng.uniform(-180, 180, n - m),
                        [4.352, 4.355, 4.358, 4.370, 4.372, 4.374, 4.40, 4.41, 4.42, 4.31, 4.33, 4.35, 4.405, 4.406]])
    y = np.concatenate([near[1] + rng.uniform(-spread, spread, m), rng.uniform(-90, 90, n - m),
                        [50.852, 50.855, 50.858, 50.852, 50.853, 50.854, 50.10, 50.11, 50.12, 50.20, 50.22, 50.24,
                         50.855, 50.856]])
    ids = [f"dev-{v:05d}" for v in rng.integers(0, 3000, len(x))]
    ids[-14:] = list("AAABBBCCCDDDEE")
    ts = np.sort(rng.integers(0, 30_000, len(x))).astype(np.int64)
    return x, y, ids, ts


@pytest.mark.parametrize("approximate", [False, True])
def test_q1_high_risk(sf, oracle_mod, approximate):
    g = sf.UniformGrid(100, *WORLD)
    og = oracle_mod.grid(100, *WORLD)
    rings = high_risk_rings()
    polys = [sf.Polygon(r, g) for r in rings]
    raw = [[[tuple(v) for v in ring] for ring in r] for r in rings]
    x, y, ids, ts = gps_points(1, 400_000, (4.355, 50.855), 0.02)
    # points on the polygon's edges and corners and at r = 0.001 +- 1 ulp from its sides
    ex = np.array([4.35, 4.36, 4.355, 4.355, 4.349, 4.361, np.nextafter(4.349, 0), np.nextafter(4.361, 9)])
    ey = np.array([50.85, 50.86, 50.849, 50.861, 50.855, 50.855, 50.855, 50.855])
    x, y = np.concatenate([x, ex]), np.concatenate([y, ey])
    ids = ids + [f"edge-{i}" for i in range(len(ex))]
    ts = np.concatenate([ts, np.full(len(ex), ts[-1])])
    op = sf.PointPolygonRangeQuery(realtime(sf, approximate), g)
    d = sf.ObjIdDict(0)
    keys = d.intern(ids)
    lo = 0
    total = 0
    for hi in (100_000, 250_001, len(x)):  # a RealTime stream: batch by batch
        w = sf.PointWindow.from_numpy(x[lo:hi], y[lo:hi], keys[lo:hi], ts[lo:hi])
        w.objid_dict = d
        res = op.run(w, polys, 0.001)
        got = res.indices().astype(np.int64)
        exp = oracle_mod.range_ppoly(og, x[lo:hi], y[lo:hi], oracle_mod.Polygons(raw), 0.001, approximate)
        np.testing.assert_array_equal(got, exp)
        assert w.objid_strings(w.objID.cpu().numpy()[got]) == [ids[lo + i] for i in got]
        total += len(got)
        lo = hi
    assert total > 1000  # the Brussels cluster's points in and around the zone


@pytest.mark.parametrize("q,r,layers", [((4.35, 50.85), 100.0, (18, 28)), ((4.3658, 50.6456), 2.0, (-1, 1))])
def test_mn_q1(sf, oracle_mod, q, r, layers):
    g = sf.UniformGrid(100, *WORLD)
    og = oracle_mod.grid(100, *WORLD)
    assert oracle_mod.layers(og, r) == layers
    x, y, ids, ts = gps_points(2, 600_000, q, 3.0)
    qp = sf.Point("query", q[0], q[1], 0, g)
    op = sf.PointPointRangeQuery(realtime(sf), g)
    d = sf.ObjIdDict(0)
    keys = d.intern(ids)
    w = sf.PointWindow.from_numpy(x, y, keys, ts)
    w.objid_dict = d
    res = op.run(w, {qp}, r)
    got = res.indices().astype(np.int64)
    exp = oracle_mod.range_pp(og, x, y, [q[0]], [q[1]], r)
    np.testing.assert_array_equal(got, exp)
    assert w.objid_strings(keys[got]) == [ids[i] for i in got]
    # MN_Q1's windowAll(TumblingEventTimeWindows.of(5 s)) count of the emitted points
    wins = np.bincount(ts[got] // 5000, minlength=6)
    exp_wins = np.bincount(ts[exp] // 5000, minlength=6)
    np.testing.assert_array_equal(wins, exp_wins)
    assert 0 < len(got) < len(x)
