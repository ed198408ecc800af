"""GPU parity: every hot-path kernel, through the C ABI, against the oracle (C restatement)
and the committed golden fixtures.  Bit-exact for cells, index/pair sets and kNN
(objID, rank) lists; kNN distances are compared with rtol 1e-12 (north star) and are in
fact bit-identical.  Run on an MI355X with `pytest -m gpu`."""
import os

import numpy as np
import pytest

from conftest import BEIJING, GOLDEN, QPOINT

pytestmark = pytest.mark.gpu


def load(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def win(sf, x, y, objID=None):
    return sf.PointWindow.from_numpy(np.asarray(x, np.float64), np.asarray(y, np.float64), objID)


def conf(sf, approximate=False, metric=0):
    c = sf.QueryConfiguration(sf.QueryType.WindowBased)
    c.setApproximateQuery(approximate)
    c.distanceMetric = metric
    return c


# ------------------------------------------------------------------ K1 cell assignment
@pytest.mark.parametrize("n", [100, 500])
def test_cells_golden(sf, n):
    f = load(f"cells_n{n}.npz")
    g = sf.UniformGrid(n, *BEIJING)
    cx, cy = sf.assign_cells(win(sf, f["x"], f["y"]), g)
    np.testing.assert_array_equal(cx.cpu().numpy(), f["cx"])
    np.testing.assert_array_equal(cy.cpu().numpy(), f["cy"])


def test_cells_random_large(sf, oracle_mod):
    """fp64 division + floor + Java (int) on 1M+ points incl. exact cell boundaries."""
    g = sf.UniformGrid(1000, *BEIJING)
    og = oracle_mod.grid(1000, *BEIJING)
    x0, y0 = oracle_mod.java_random_points(3, 1_000_001, 115.0, 118.2, 39.0, 41.7)
    cl = og.cellLength
    bx = 115.5 + np.arange(1001) * cl  # points on (and one ulp around) every cell edge
    by = 39.6 + np.arange(1001) * cl
    x = np.concatenate([x0, bx, np.nextafter(bx, -np.inf), np.nextafter(bx, np.inf), [np.nan, np.inf, -1e300]])
    y = np.concatenate([y0, by, np.nextafter(by, np.inf), np.nextafter(by, -np.inf), [40.0, np.nan, 1e300]])
    cx, cy = sf.assign_cells(win(sf, x, y), g)
    ocx, ocy = oracle_mod.assign_cells(og, x, y)
    np.testing.assert_array_equal(cx.cpu().numpy(), ocx)
    np.testing.assert_array_equal(cy.cpu().numpy(), ocy)


def test_cells_odd_sizes(sf, oracle_mod):
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    for n in (1, 2, 3, 63, 64, 65, 129):
        x, y = oracle_mod.java_random_points(n, n, *BEIJING)
        cx, cy = sf.assign_cells(win(sf, x, y), g)
        ocx, ocy = oracle_mod.assign_cells(og, x, y)
        np.testing.assert_array_equal(cx.cpu().numpy(), ocx)
        np.testing.assert_array_equal(cy.cpu().numpy(), ocy)


# ------------------------------------------------------------------ K2 bucketing
def bucket_expected(oracle_mod, og, gn, x, y):
    """keyBy(gridID) restated: bucket = valid cell cy*n + cx (out-of-grid last), points of a
    bucket in arrival order (a stable sort of the keys) -- the exact permutation."""
    cx, cy = oracle_mod.assign_cells(og, x, y)
    valid = (cx >= 0) & (cy >= 0) & (cx < gn) & (cy < gn)
    key = np.where(valid, cy.astype(np.int64) * gn + cx, gn * gn)
    perm = np.argsort(key, kind="stable")
    start = np.searchsorted(key[perm], np.arange(gn * gn + 2), side="left")
    return perm, start


@pytest.mark.parametrize("gn,n,box,clustered", [
    (100, 200_001, (115.3, 117.8, 39.5, 41.2), False),     # 14-bit keys: 2 passes, out-of-grid points
    (1000, 1_500_000, BEIJING, False),                      # 20-bit keys: 2 passes
    (2048, 700_000, BEIJING, True),                         # 23-bit keys: 3 passes, hot spots
    (7, 5_000, BEIJING, True),                              # 1 pass
    (500, 1, BEIJING, False), (500, 63, BEIJING, False), (500, 4097, BEIJING, True),
    # row mode (gn <= 511): the most rows, out-of-grid points; mostly empty rows
    (511, 800_000, (115.3, 117.8, 39.5, 41.2), True), (300, 100, BEIJING, False),
    (23, 50, (115.3, 117.8, 39.5, 41.2), False),            # the smallest two-pass grid: fewer points than rows
    (64, 70_000, (116.39, 116.41, 39.5, 41.2), False),      # one column: every row one cell
    # r06 whole-row sort (radix_row_sort_kernel): the bench window (~20K-point rows), and rows
    # around the one-segment bound (32768: some rows sorted whole, the others by segments)
    (500, 10_000_000, BEIJING, False), (100, 2_340_500, BEIJING, False),  # (71.4 occupied rows)
])
def test_bucket_by_cell_exact(sf, oracle_mod, gn, n, box, clustered):
    g = sf.UniformGrid(gn, *BEIJING)
    og = oracle_mod.grid(gn, *BEIJING)
    x, y = oracle_mod.java_random_points(9 + gn, n, *box)
    if clustered:  # Gaussian hot spots, sigma 0.01 deg: most points in a few cells
        rng = np.random.default_rng(gn)
        c = rng.integers(0, 4, n)
        cxs, cys = np.array([116.0, 116.4, 117.1, 115.9]), np.array([39.9, 40.3, 40.0, 40.8])
        h = rng.random(n) < 0.8
        x = np.where(h, cxs[c] + 0.01 * rng.standard_normal(n), x)
        y = np.where(h, cys[c] + 0.01 * rng.standard_normal(n), y)
    perm, start = sf.bucket_by_cell(win(sf, x, y), g)
    perm = perm.cpu().numpy().view(np.uint32).astype(np.int64)
    start = start.cpu().numpy().view(np.uint32).astype(np.int64)
    ep, es = bucket_expected(oracle_mod, og, gn, x, y)
    np.testing.assert_array_equal(perm, ep)
    np.testing.assert_array_equal(start, es)


@pytest.mark.parametrize("rowsort", ["0", "1"])
def test_bucket_row_sort_matches_segments(sf, oracle_mod, rowsort, monkeypatch):
    """GF_K2_ROWSORT=0 (A/B knob: every row by segments) and the default whole-row sort give the
    same exact permutation on a clustered window with one- and multi-segment rows."""
    monkeypatch.setenv("GF_K2_ROWSORT", rowsort)
    gn, n = 200, 2_000_000
    g = sf.UniformGrid(gn, *BEIJING)
    og = oracle_mod.grid(gn, *BEIJING)
    x, y = oracle_mod.java_random_points(5, n, *BEIJING)
    rng = np.random.default_rng(1)
    h = rng.random(n) < 0.3
    y = np.where(h, 40.3 + 0.002 * rng.standard_normal(n), y)  # two hot rows: multi-segment
    perm, start = sf.bucket_by_cell(win(sf, x, y), g)
    ep, es = bucket_expected(oracle_mod, og, gn, x, y)
    np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32).astype(np.int64), ep)
    np.testing.assert_array_equal(start.cpu().numpy().view(np.uint32).astype(np.int64), es)


@pytest.mark.parametrize("gn", [500, 2048])
def test_bucket_by_cell_one_row_nan(sf, oracle_mod, gn):
    """One row holding most points (row mode: ~10 segments chained in one row's scan; the LSD
    path at gn = 2048), NaN / inf coordinates (out-of-grid bucket), points on cell bounds."""
    g = sf.UniformGrid(gn, *BEIJING)
    og = oracle_mod.grid(gn, *BEIJING)
    n = 350_000
    x, y = oracle_mod.java_random_points(77, n, *BEIJING)
    y = np.where(np.arange(n) % 7 != 0, 40.31, y)  # 6/7 of the points in one row
    x[::1001] = np.nan
    y[5::997] = np.inf
    cl = (BEIJING[1] - BEIJING[0]) / gn
    x[3::501] = BEIJING[0] + cl * (np.arange(3, n, 501) % gn)  # exactly on column bounds
    perm, start = sf.bucket_by_cell(win(sf, x, y), g)
    perm = perm.cpu().numpy().view(np.uint32).astype(np.int64)
    start = start.cpu().numpy().view(np.uint32).astype(np.int64)
    ep, es = bucket_expected(oracle_mod, og, gn, x, y)
    np.testing.assert_array_equal(perm, ep)
    np.testing.assert_array_equal(start, es)


def test_bucket_by_cell_empty_and_repeatable(sf, oracle_mod):
    g = sf.UniformGrid(50, *BEIJING)
    import torch
    w = sf.PointWindow(torch.empty(0, dtype=torch.float64, device="cuda"), torch.empty(0, dtype=torch.float64, device="cuda"),
                       torch.empty(0, dtype=torch.int64, device="cuda"), torch.empty(0, dtype=torch.int64, device="cuda"))
    perm, start = sf.bucket_by_cell(w, g)
    assert start.cpu().numpy().sum() == 0 and start.numel() == 50 * 50 + 2
    x, y = oracle_mod.java_random_points(4, 333_333, *BEIJING)
    a = sf.bucket_by_cell(win(sf, x, y), g)[0].cpu().numpy()
    b = sf.bucket_by_cell(win(sf, x, y), g)[0].cpu().numpy()
    np.testing.assert_array_equal(a, b)


# ------------------------------------------------------------------ range point-point
def test_range_pp_golden(sf):
    f = load("range_pp.npz")
    g = sf.UniformGrid(100, *BEIJING)
    w = win(sf, f["x"], f["y"])
    for qn in ("q1", "q3"):
        qs = [sf.Point(str(i), a, b, 0, g) for i, (a, b) in enumerate(zip(f[f"{qn}_qx"], f[f"{qn}_qy"]))]
        for r in (0.5, 0.05, 0.02, 0.0):
            for ap in (0, 1):
                res = sf.PointPointRangeQuery(conf(sf, bool(ap)), g).run(w, qs, r)
                exp = f[f"{qn}_r{r}_a{ap}"]
                np.testing.assert_array_equal(res.multiset_indices(), exp, err_msg=f"{qn} r={r} ap={ap}")
                assert res.count() == len(np.unique(exp))
                assert res.multiset_size() == len(exp)


@pytest.mark.parametrize("r,n", [(0.5, 100), (0.05, 100), (0.02, 500), (0.3, 500), (0.0011, 1000)])
def test_range_pp_large(sf, oracle_mod, r, n):
    g = sf.UniformGrid(n, *BEIJING)
    og = oracle_mod.grid(n, *BEIJING)
    x, y = oracle_mod.java_random_points(17, 1_000_003, 115.4, 117.7, 39.5, 41.2)
    w = win(sf, x, y)
    q = sf.Point("q", *QPOINT, 0, g)
    res = sf.PointPointRangeQuery(conf(sf), g).run(w, [q], r)
    exp = oracle_mod.range_pp(og, x, y, [QPOINT[0]], [QPOINT[1]], r)
    np.testing.assert_array_equal(res.indices().astype(np.int64), exp)


def test_range_pp_multi_query_large(sf, oracle_mod):
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    x, y = oracle_mod.java_random_points(21, 400_000, *BEIJING)
    qx, qy = oracle_mod.java_random_points(22, 25, 115.4, 117.7, 39.5, 41.2)
    w = win(sf, x, y)
    qs = [sf.Point(str(i), a, b, 0, g) for i, (a, b) in enumerate(zip(qx, qy))]
    for r in (0.05, 0.11, 0.01):
        for ap in (False, True):
            res = sf.PointPointRangeQuery(conf(sf, ap), g).run(w, qs, r)
            exp = oracle_mod.range_pp(og, x, y, qx, qy, r, ap)
            np.testing.assert_array_equal(res.multiset_indices(), exp)


def test_range_pp_edge_windows(sf, oracle_mod):
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointRangeQuery(conf(sf), g)
    # empty window
    res = op.run(win(sf, np.zeros(0), np.zeros(0)), [q], 0.5)
    assert res.count() == 0 and len(res.indices()) == 0
    # every point exactly at the query point / on the r boundary / NaN / inf
    r = 0.5
    x = np.array([QPOINT[0], QPOINT[0] + r, QPOINT[0], np.nan, np.inf, 115.5, 117.6, QPOINT[0] - r])
    y = np.array([QPOINT[1], QPOINT[1], QPOINT[1] + r, 40.0, 40.0, 39.6, 41.1, QPOINT[1]])
    for n in range(1, len(x) + 1):
        res = op.run(win(sf, x[:n], y[:n]), [q], r)
        np.testing.assert_array_equal(res.indices().astype(np.int64),
                                      oracle_mod.range_pp(og, x[:n], y[:n], [QPOINT[0]], [QPOINT[1]], r))


def test_range_query_cell_out_of_grid(sf, oracle_mod):
    """g == 0 adds the (out-of-grid) query cell without validKey (UniformGrid.java:171-174)."""
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    qx, qy = 115.48, 40.0  # cell -1
    x, y = oracle_mod.java_random_points(5, 100_000, 115.3, 115.7, 39.8, 40.2)
    res = sf.PointPointRangeQuery(conf(sf), g).run(win(sf, x, y), [sf.Point("q", qx, qy, 0, g)], 0.05)
    np.testing.assert_array_equal(res.indices().astype(np.int64), oracle_mod.range_pp(og, x, y, [qx], [qy], 0.05))


# ------------------------------------------------------------------ range point-polygon
def golden_polygons(sf, f, g):
    polys = []
    ro, vo, vx, vy = f["ring_off"], f["vert_off"], f["vx"], f["vy"]
    for p in range(len(ro) - 1):
        rings = [list(zip(vx[vo[j]:vo[j + 1]], vy[vo[j]:vo[j + 1]])) for j in range(ro[p], ro[p + 1])]
        polys.append(sf.Polygon(rings, g))
    return polys


def test_range_ppoly_golden(sf):
    f = load("range_ppoly.npz")
    g = sf.UniformGrid(100, *BEIJING)
    polys = golden_polygons(sf, f, g)
    w = win(sf, f["x"], f["y"])
    for r in (0.001, 0.05, 0.3):
        for ap in (0, 1):
            res = sf.PointPolygonRangeQuery(conf(sf, bool(ap)), g).run(w, polys, r)
            np.testing.assert_array_equal(res.indices().astype(np.int64), f[f"r{r}_a{ap}"], err_msg=f"r={r} ap={ap}")


@pytest.mark.parametrize("n,r", [(100, 0.001), (500, 0.001), (100, 0.05)])
def test_range_ppoly_generated_1000(sf, oracle_mod, n, r):
    """C3 shape (1000 generateQueryPolygons squares) at a test-sized window."""
    g = sf.UniformGrid(n, *BEIJING)
    og = oracle_mod.grid(n, *BEIJING)
    raw = oracle_mod.generate_query_polygons(1000, 115.5, 39.6, 117.6, 41.1)
    polys = [sf.Polygon(p, g) for p in raw]
    x, y = oracle_mod.java_random_points(31, 150_000, 115.45, 115.75, *BEIJING[2:])
    w = win(sf, x, y)
    for ap in (False, True):
        res = sf.PointPolygonRangeQuery(conf(sf, ap), g).run(w, polys, r)
        exp = oracle_mod.range_ppoly(og, x, y, oracle_mod.Polygons(raw), r, ap)
        np.testing.assert_array_equal(res.indices().astype(np.int64), exp)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_range_table_defer_modes(sf, oracle_mod, mode):
    """Table-mode candidate tests inline (1), deferred (2) and deferred behind the span
    prefilter (3, the C3 default: the stream only rules out points outside the class spans, the
    block classifies the rest with the table at its end): the 1000 generateQueryPolygons squares
    with points across the whole grid, NaN and outside-the-grid points; a many-point query set."""
    n = 500
    g = sf.UniformGrid(n, *BEIJING)
    og = oracle_mod.grid(n, *BEIJING)
    raw = oracle_mod.generate_query_polygons(1000, 115.5, 39.6, 117.6, 41.1)
    polys = [sf.Polygon(p, g) for p in raw]
    x, y = oracle_mod.java_random_points(33, 400_000, 115.4, 117.7, 39.5, 41.2)
    x[:5] = np.nan
    y[5:10] = np.nan
    x[10:20] = BEIJING[0] - 1e-3
    w = win(sf, x, y)
    for ap in (False, True):
        op = sf.PointPolygonRangeQuery(conf(sf, ap), g)
        op.tuning = (0, mode)
        res = op.run(w, polys, 0.001)
        exp = oracle_mod.range_ppoly(og, x, y, oracle_mod.Polygons(raw), 0.001, ap)
        np.testing.assert_array_equal(res.indices().astype(np.int64), exp, err_msg=f"ap={ap}")
        assert res.count() == len(exp)
    qx, qy = oracle_mod.java_random_points(34, 300, 115.5, 115.6, 40.0, 40.4)
    op = sf.PointPointRangeQuery(conf(sf), g)
    op.tuning = (0, mode)
    res = op.run(w, [sf.Point(str(i), qx[i], qy[i], 0, g) for i in range(len(qx))], 0.004)
    exp = oracle_mod.range_pp(og, x, y, qx, qy, 0.004)
    np.testing.assert_array_equal(res.indices().astype(np.int64), exp)


@pytest.mark.parametrize("lanes", [1, 3, 37, 63])
def test_range_drain_partial_waves(sf, oracle_mod, lanes):
    """The block-end candidate drain (drain_own_queue, DEFER 1 and 3) run by only the first
    `lanes` lanes of every wave (gf_range_plan_set_drain_lanes): its points come from a block
    cursor taken by the active lanes, groups form among them and a point's hit is recorded by the
    lowest active lane of its group that found it -- identical results for any exec mask
    (safe by construction, not by its calling context).  The C3 shape
    (generateQueryPolygons squares, PointPolygonRangeQuery.java:170-204) and a point query set."""
    n = 500
    g = sf.UniformGrid(n, *BEIJING)
    og = oracle_mod.grid(n, *BEIJING)
    raw = oracle_mod.generate_query_polygons(1000, 115.5, 39.6, 117.6, 41.1)
    polys = [sf.Polygon(p, g) for p in raw]
    x, y = oracle_mod.java_random_points(35, 600_000, 115.4, 117.7, 39.5, 41.2)
    x[:5] = np.nan
    w = win(sf, x, y)
    exp = oracle_mod.range_ppoly(og, x, y, oracle_mod.Polygons(raw), 0.001)
    for mode in (1, 3):
        op = sf.PointPolygonRangeQuery(conf(sf), g)
        op.tuning = (0, mode)
        op.drain_lanes = lanes
        res = op.run(w, polys, 0.001)
        np.testing.assert_array_equal(res.indices().astype(np.int64), exp, err_msg=f"mode {mode}")
        assert res.count() == len(exp)
    qx, qy = oracle_mod.java_random_points(36, 300, 115.5, 115.6, 40.0, 40.4)
    op = sf.PointPointRangeQuery(conf(sf), g)
    op.tuning = (0, 3)
    op.drain_lanes = lanes
    res = op.run(w, [sf.Point(str(i), qx[i], qy[i], 0, g) for i in range(len(qx))], 0.004)
    np.testing.assert_array_equal(res.indices().astype(np.int64), oracle_mod.range_pp(og, x, y, qx, qy, 0.004))


def _ulps(v, k):
    for _ in range(abs(k)):
        v = np.nextafter(v, np.inf if k > 0 else -np.inf)
    return float(v)


def test_range_ppoly_inside_cells_and_edges(sf, oracle_mod):
    """Exact-mode shortcuts of the point-polygon plan: candidate cells wholly inside an
    axis-aligned rectangle are accepted untested (kInside), candidate points go through the
    deferred queue with envelope pruning.  Rectangles whose edges sit on / a few ulps off
    cell boundaries, a rectangle with a hole (not kInside), a diamond, a triangle; points on
    edges, at cell thresholds, NaN."""
    n = 100
    g = sf.UniformGrid(n, *BEIJING)
    og = oracle_mod.grid(n, *BEIJING)
    cl = (BEIJING[1] - BEIJING[0]) / n
    bx = lambda c, k=0: _ulps(BEIJING[0] + c * cl, k)
    by = lambda c, k=0: _ulps(BEIJING[2] + c * cl, k)
    raw = []
    for i, (k0, k1) in enumerate([(0, 0), (1, -1), (-1, 1), (2, -3), (-2, 2)]):
        x1, x2, y1, y2 = bx(10 + 7 * i, k0), bx(14 + 7 * i, k1), by(20, k0), by(25, k1)
        raw.append([[(x1, y1), (x2, y1), (x2, y2), (x1, y2), (x1, y1)]])
    # rectangle with a rectangular hole
    raw.append([[(bx(50), by(30)), (bx(56), by(30)), (bx(56), by(36)), (bx(50), by(36)), (bx(50), by(30))],
                [(bx(52), by(32)), (bx(54), by(32)), (bx(54), by(34)), (bx(52), by(34)), (bx(52), by(32))]])
    # diamond and triangle
    cx0, cy0, h = bx(70), by(40), 3 * cl
    raw.append([[(cx0, cy0 - h), (cx0 + h, cy0), (cx0, cy0 + h), (cx0 - h, cy0), (cx0, cy0 - h)]])
    raw.append([[(bx(80), by(10)), (bx(88), by(10)), (bx(84), by(18)), (bx(80), by(10))]])
    # rectangle given clockwise, starting at another corner
    raw.append([[(bx(30, 1), by(50)), (bx(30, 1), by(46)), (bx(26), by(46)), (bx(26), by(50)), (bx(30, 1), by(50))]])
    # adjacent rectangles sharing an edge inside a cell (their union covers it), and a pair
    # separated by a 2-ulp gap (never covered)
    mid, m2 = bx(40) + 0.4 * cl, bx(46) + 0.6 * cl
    for (a0, a1, b0, b1) in [(bx(40), mid, mid, bx(44)), (bx(46), m2, _ulps(m2, 2), bx(50))]:
        raw.append([[(a0, by(20)), (a1, by(20)), (a1, by(24)), (a0, by(24)), (a0, by(20))]])
        raw.append([[(b0, by(20)), (b1, by(20)), (b1, by(24)), (b0, by(24)), (b0, by(20))]])
    polys = [sf.Polygon(p, g) for p in raw]
    x, y = oracle_mod.java_random_points(77, 300_000, BEIJING[0], bx(92), BEIJING[2], by(60))
    ex, ey = [], []
    for p in raw:
        for ring in p:
            for (ax, ay), (bx_, by_) in zip(ring[:-1], ring[1:]):
                for t in np.linspace(0.0, 1.0, 9):
                    ex.append(ax + t * (bx_ - ax))
                    ey.append(ay + t * (by_ - ay))
                for k in (-2, -1, 1, 2):
                    ex.append(_ulps(ax, k))
                    ey.append(ay)
                    ex.append(ax)
                    ey.append(_ulps(ay, k))
    for c in range(8, 60):
        for k in (-1, 0, 1):
            ex.append(bx(c, k))
            ey.append(by(22, 0) + 0.0003)
            ex.append(bx(12) + 0.0002)
            ey.append(by(c, k))
    ex += [np.nan, bx(12), np.nan, bx(52) + 1e-4, _ulps(m2, 1), m2, _ulps(m2, 2), mid]
    ey += [by(22), np.nan, np.nan, by(33), by(22), by(22), by(22), by(22)]
    x = np.concatenate([np.asarray(ex), x])
    y = np.concatenate([np.asarray(ey), y])
    w = win(sf, x, y)
    for r in (0.0, 0.0005, 0.001, 0.02):
        for ap in (False, True):
            res = sf.PointPolygonRangeQuery(conf(sf, ap), g).run(w, polys, r)
            exp = oracle_mod.range_ppoly(og, x, y, oracle_mod.Polygons(raw), r, ap)
            np.testing.assert_array_equal(res.indices().astype(np.int64), exp, err_msg=f"r={r} ap={ap}")
            assert res.count() == len(exp)


# ------------------------------------------------------------------ kNN
def check_knn(res, oo, od, oi):
    np.testing.assert_array_equal(res.objID, oo)
    np.testing.assert_array_equal(res.idx, oi)
    np.testing.assert_allclose(res.dist, od, rtol=1e-12, atol=0)
    np.testing.assert_array_equal(res.dist, od)  # in fact bit-identical


def test_knn_golden(sf):
    f = load("knn.npz")
    g = sf.UniformGrid(100, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    for tag, ob in (("u", f["objID"]), ("d", f["objID_dup"])):
        w = win(sf, f["x"], f["y"], ob)
        for r in (0.5, 0.05, 0.3):
            for k in (1, 50, 100):
                res = sf.PointPointKNNQuery(conf(sf), g).run(w, q, r, k)
                check_knn(res, f[f"{tag}_r{r}_k{k}_obj"], f[f"{tag}_r{r}_k{k}_d"], f[f"{tag}_r{r}_k{k}_idx"])


@pytest.mark.parametrize("n,r,k", [(500, 0.5, 50), (500, 0.05, 50), (1000, 0.5, 100), (100, 0.3, 7)])
def test_knn_large_sampled(sf, oracle_mod, n, r, k):
    """Windows >= 1M points take the sample -> threshold -> scan -> select path."""
    g = sf.UniformGrid(n, *BEIJING)
    og = oracle_mod.grid(n, *BEIJING)
    N = 2_000_001
    x, y = oracle_mod.java_random_points(n + k, N, *BEIJING)
    obj = np.random.default_rng(k).permutation(N).astype(np.int64)
    q = sf.Point("q", *QPOINT, 0, g)
    res = sf.PointPointKNNQuery(conf(sf), g).run(win(sf, x, y, obj), q, r, k)
    st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
    check_knn(res, oo, od, oi)


def test_knn_duplicate_objids_sampled(sf, oracle_mod):
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    N = 1_500_000
    x, y = oracle_mod.java_random_points(77, N, *BEIJING)
    obj = (np.arange(N) % 997).astype(np.int64)  # each objID ~1500 times (trajectories)
    q = sf.Point("q", *QPOINT, 0, g)
    for k in (50, 300, 512):  # 512: the largest device k, chunked general select path
        res = sf.PointPointKNNQuery(conf(sf), g).run(win(sf, x, y, obj), q, 0.5, k)
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
        check_knn(res, oo, od, oi)


def test_knn_forced_fallback(sf, oracle_mod):
    """Candidate-buffer overflow -> exact partitioned fallback."""
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    x, y = oracle_mod.java_random_points(8, 300_000, *BEIJING)
    obj = np.arange(len(x), dtype=np.int64)[::-1].copy()
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    w = win(sf, x, y, obj)
    op.set_capacity(w.x.device.index, q, 0.5, 50, 4096)
    res = op.run(w, q, 0.5, 50)
    st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, 50)
    check_knn(res, oo, od, oi)


def test_knn_ties_broken_by_objid(sf, oracle_mod):
    """Points at identical distances: ranks follow objID (build contract, Appendix A7)."""
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    base_x, base_y = oracle_mod.java_random_points(4, 2000, 116.3, 116.5, 39.85, 40.0)
    x = np.repeat(base_x, 8)
    y = np.repeat(base_y, 8)
    obj = np.random.default_rng(0).permutation(len(x)).astype(np.int64)
    q = sf.Point("q", *QPOINT, 0, g)
    res = sf.PointPointKNNQuery(conf(sf), g).run(win(sf, x, y, obj), q, 0.5, 100)
    st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, 100)
    check_knn(res, oo, od, oi)


def test_knn_hypot_metric(sf, oracle_mod):
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    x, y = oracle_mod.java_random_points(12, 1_200_000, *BEIJING)
    obj = np.arange(len(x), dtype=np.int64)
    q = sf.Point("q", *QPOINT, 0, g)
    res = sf.PointPointKNNQuery(conf(sf, metric=1), g).run(win(sf, x, y, obj), q, 0.5, 50)
    st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, 50, metric=1)
    check_knn(res, oo, od, oi)


def test_knn_edge_windows(sf, oracle_mod):
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    assert len(op.run(win(sf, np.zeros(0), np.zeros(0), np.zeros(0, np.int64)), q, 0.5, 50)) == 0
    x = np.array([QPOINT[0], np.nan, QPOINT[0] + 0.5, 117.0, QPOINT[0] + 0.1])
    y = np.array([QPOINT[1], 40.0, QPOINT[1], 41.0, QPOINT[1]])
    obj = np.array([5, 4, 3, 2, 1], np.int64)
    for k in (1, 2, 3, 10):
        res = op.run(win(sf, x, y, obj), q, 0.5, k)
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
        check_knn(res, oo, od, oi)


def test_knn_merge_dev_equals_single_window(sf, oracle_mod):
    """Per-shard records merged on the device == the whole window (the multi-GPU funnel)."""
    import torch

    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    x, y = oracle_mod.java_random_points(55, 400_000, *BEIJING)
    obj = np.random.default_rng(1).permutation(len(x)).astype(np.int64)
    q = sf.Point("q", *QPOINT, 0, g)
    k = 64
    op = sf.PointPointKNNQuery(conf(sf), g)
    rb = sf.spatialOperators.knn_record_bytes(k)
    shards = np.array_split(np.arange(len(x)), 4)
    recs = torch.zeros(4 * rb, dtype=torch.uint8, device="cuda")
    for s, ix in enumerate(shards):
        w = win(sf, x[ix], y[ix], obj[ix])
        op.enqueue(w, q, 0.5, k, recs[s * rb:(s + 1) * rb])
    # shard-local indices -> global
    torch.cuda.synchronize()
    host = recs.cpu().numpy().tobytes()
    fixed = bytearray(host)
    for s, ix in enumerate(shards):
        st, o, d, i = sf.spatialOperators.decode_knn_record(host[s * rb:(s + 1) * rb], k)
        assert st == 0
        i = i + ix[0]
        off = s * rb + 32 + 16 * k
        fixed[off:off + 8 * len(i)] = i.astype(np.int64).tobytes()
    recs_dev = torch.frombuffer(bytearray(fixed), dtype=torch.uint8).cuda()
    out = torch.zeros(rb, dtype=torch.uint8, device="cuda")
    import ctypes as C
    from spatialflink_amd import _lib

    ctx = _lib.context(0)
    _lib.check(_lib.lib().gf_knn_merge_dev(ctx.handle, k, recs_dev.data_ptr(), 4, out.data_ptr()), ctx.handle, "merge")
    st, oo2, od2, oi2 = sf.spatialOperators.decode_knn_record(out.cpu().numpy().tobytes(), k)
    st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
    np.testing.assert_array_equal(oo2, oo)
    np.testing.assert_array_equal(od2, od)
    np.testing.assert_array_equal(oi2, oi)


def test_knn_deterministic(sf):
    g = sf.UniformGrid(500, *BEIJING)
    x, y = sf.synthetic_uniform(42, 2_000_000, *BEIJING)
    w = win(sf, x, y, np.arange(len(x), dtype=np.int64))
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    a = op.run(w, q, 0.5, 50)
    for _ in range(3):
        b = op.run(w, q, 0.5, 50)
        np.testing.assert_array_equal(a.objID, b.objID)
        np.testing.assert_array_equal(a.dist, b.dist)


# ------------------------------------------------------------------ join
def test_join_golden(sf):
    f = load("join.npz")
    g = sf.UniformGrid(100, *BEIJING)
    wo, wq = win(sf, f["ox"], f["oy"]), win(sf, f["qx"], f["qy"])
    for r in (0.001, 0.05, 0.0):
        for ap in (0, 1):
            if r == 0.0 and ap:
                continue
            got = sf.PointPointJoinQuery(conf(sf, bool(ap)), g, g).run(wo, wq, r)
            np.testing.assert_array_equal(got, f[f"r{r}_a{ap}"], err_msg=f"r={r} ap={ap}")


@pytest.mark.parametrize("n,r", [(1000, 0.001), (500, 0.01), (100, 0.03)])
def test_join_large(sf, oracle_mod, n, r):
    g = sf.UniformGrid(n, *BEIJING)
    og = oracle_mod.grid(n, *BEIJING)
    ox, oy = oracle_mod.java_random_points(61, 300_000, 115.4, 117.7, 39.5, 41.2)
    qx, qy = oracle_mod.java_random_points(62, 30_000, 115.4, 117.7, 39.5, 41.2)
    got = sf.PointPointJoinQuery(conf(sf), g, g).run(win(sf, ox, oy), win(sf, qx, qy), r)
    st, pairs = oracle_mod.join_pp(og, og, ox, oy, qx, qy, r)
    exp = np.array(sorted(map(tuple, pairs.tolist())), np.int64).reshape(-1, 2)
    np.testing.assert_array_equal(got, exp)


def test_join_negative_radius_raises(sf):
    g = sf.UniformGrid(100, *BEIJING)
    w = win(sf, [116.0], [40.0])
    with pytest.raises(sf._lib.CandidateLayersError):
        sf.PointPointJoinQuery(conf(sf), g, g).run(w, w, -0.5)


def test_join_different_query_grid(sf, oracle_mod):
    ug = sf.UniformGrid(100, *BEIJING)
    qg = sf.UniformGrid(80, 115.4, 117.8, 39.5, 41.3)
    oug, oqg = oracle_mod.grid(100, *BEIJING), oracle_mod.grid(80, 115.4, 117.8, 39.5, 41.3)
    ox, oy = oracle_mod.java_random_points(71, 50_000, *BEIJING)
    qx, qy = oracle_mod.java_random_points(72, 5_000, *BEIJING)
    got = sf.PointPointJoinQuery(conf(sf), ug, qg).run(win(sf, ox, oy), win(sf, qx, qy), 0.02)
    st, pairs = oracle_mod.join_pp(oug, oqg, ox, oy, qx, qy, 0.02)
    exp = np.array(sorted(map(tuple, pairs.tolist())), np.int64).reshape(-1, 2)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("n,r,qn,qbox", [(100, 0.001, 100, None), (100, 0.05, 100, None),
                                          (200, 0.012, 150, (115.3, 117.9, 39.4, 41.4)),
                                          (100, 0.05, 100, (115.45, 117.65, 39.55, 41.15))])
def test_join_row_path_edges(sf, oracle_mod, n, r, qn, qbox):
    """Row-bucketed join vs the legacy probe vs the oracle: points outside the grid on both
    sides (clamped query rows / columns need the true-cell test), NaN coordinates, a
    query grid different from the ordinary grid, c = 1..3."""
    from spatialflink_amd import _lib

    ug = sf.UniformGrid(n, *BEIJING)
    qgb = qbox or BEIJING
    qg = sf.UniformGrid(qn, *qgb)
    oug, oqg = oracle_mod.grid(n, *BEIJING), oracle_mod.grid(qn, *qgb)
    ox, oy = oracle_mod.java_random_points(81, 120_000, 115.3, 117.8, 39.4, 41.3)
    qx, qy = oracle_mod.java_random_points(82, 40_000, 115.3, 117.8, 39.4, 41.3)
    ox[:3] = np.nan
    qy[5:8] = np.nan
    qx[10:40] = BEIJING[0] - np.linspace(0, 0.02, 30)  # just left of the grid
    qy[40:70] = BEIJING[3] + np.linspace(0, 0.02, 30)  # just above
    st, pairs = oracle_mod.join_pp(oug, oqg, ox, oy, qx, qy, r)
    exp = np.array(sorted(map(tuple, pairs.tolist())), np.int64).reshape(-1, 2)
    ctx = _lib.context(0)
    for legacy in (0, 1):
        _lib.check(_lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_JOIN_LEGACY, legacy), ctx.handle, "flag")
        try:
            got = sf.PointPointJoinQuery(conf(sf), ug, qg).run(win(sf, ox, oy), win(sf, qx, qy), r)
        finally:
            _lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_JOIN_LEGACY, 0)
        np.testing.assert_array_equal(got, exp, err_msg=f"legacy={legacy}")


@pytest.mark.parametrize("n,r,metric", [(1000, 0.001, 0), (100, 0.0069, 0), (100, 0.0052, 1), (300, 0.0034, 0),
                                         (300, 0.0034, 1)])
def test_join_fine_subcells(sf, oracle_mod, n, r, metric):
    """The row path's sub-cell variant (c == 1, cl/f > r: f = 2, 3, 4) against the cell
    variant (GF_FLAG_JOIN_COARSE) and the oracle: r just below cl/f, pairs straddling cell and
    sub-cell bounds (points on the bounds, +-1 ulp, partners at r (1 - 1e-15) across them),
    edge cells, NaN and outside-the-grid points on both sides."""
    from spatialflink_amd import _lib

    g = sf.UniformGrid(n, *BEIJING)
    og = oracle_mod.grid(n, *BEIJING)
    cl = (BEIJING[1] - BEIJING[0]) / n
    f = 4 if cl / 4 > r else (3 if cl / 3 > r else 2)
    ox, oy = oracle_mod.java_random_points(101, 150_000, 115.45, 117.65, 39.55, 41.15)
    qx, qy = oracle_mod.java_random_points(102, 40_000, 115.45, 117.65, 39.55, 41.15)
    rng = np.random.default_rng(7)
    k = rng.integers(0, n * f, 4000)
    bx = BEIJING[0] + k * (cl / f)  # sub-cell and cell bounds
    by = BEIJING[2] + rng.integers(0, n * f, 4000) * (cl / f)
    bx = np.where(rng.random(4000) < 0.5, np.nextafter(bx, np.inf), np.nextafter(bx, -np.inf))
    ox[:4000], oy[:4000] = bx, by
    ang = rng.random(4000) * 2 * np.pi
    qx[:4000] = bx + r * (1 - 1e-15) * np.cos(ang)
    qy[:4000] = by + r * (1 - 1e-15) * np.sin(ang)
    qx[4000:4400], qy[4000:4400] = bx[:400] + r * (1 - 1e-15), by[:400]  # axis-aligned partners
    ox[5000:5003] = np.nan
    qy[5000:5003] = np.nan
    qx[6000:6030] = BEIJING[0] - np.linspace(0, 0.02, 30)
    ox[6000:6030] = BEIJING[0] + np.linspace(0, 0.0005, 30)
    st, pairs = oracle_mod.join_pp(og, og, ox, oy, qx, qy, r, metric=metric)
    assert st == 0 and len(pairs) > 4000
    exp = np.array(sorted(map(tuple, pairs.tolist())), np.int64).reshape(-1, 2)
    ctx = _lib.context(0)
    # the fine path, the cell path, and the streaming experiment (GF_FLAG_JOIN_STREAM: only the
    # query side bucketed, the ordinary points probed in input order)
    for coarse, stream in ((0, 0), (1, 0), (0, 1)):
        _lib.check(_lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_JOIN_COARSE, coarse), ctx.handle, "flag")
        _lib.check(_lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_JOIN_STREAM, stream), ctx.handle, "flag")
        try:
            got = sf.PointPointJoinQuery(conf(sf, False, metric), g, g).run(win(sf, ox, oy), win(sf, qx, qy), r)
        finally:
            _lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_JOIN_COARSE, 0)
            _lib.lib().gf_ctx_set_flag(ctx.handle, _lib.FLAG_JOIN_STREAM, 0)
        np.testing.assert_array_equal(got, exp, err_msg=f"coarse={coarse} stream={stream} f={f}")


def test_join_async_matches_sync(sf, oracle_mod):
    """gf_join_pp_async: consecutive windows queued without a host wait, counts in device
    memory -- the same pairs and counts as gf_join_pp; a window past the capacity reports its
    count (> cap); r == 0 takes the synchronous path and still stores the count."""
    import ctypes as C

    import torch
    from spatialflink_amd import _lib

    L = _lib.lib()
    g = sf.UniformGrid(500, *BEIJING)
    ctx = _lib.context(0)
    wins = []
    for j in range(3):
        ox, oy = oracle_mod.java_random_points(110 + j, 200_000, *BEIJING)
        qx, qy = oracle_mod.java_random_points(120 + j, 40_000, *BEIJING)
        wins.append((win(sf, ox, oy), win(sf, qx, qy)))
    for r in (0.002, 0.01):
        exp = []
        for wo, wq in wins:
            exp.append(sf.PointPointJoinQuery(conf(sf), g, g).run(wo, wq, r))
        cap = max(len(e) for e in exp) + 16
        bufs = [torch.zeros(2 * cap, dtype=torch.int32, device="cuda") for _ in wins]
        totals = torch.zeros(len(wins), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        for j, (wo, wq) in enumerate(wins):
            po, pq = wo.c_struct(), wq.c_struct()
            _lib.check(L.gf_join_pp_async(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), r,
                                          0, 0, bufs[j].data_ptr(), cap, totals[j].data_ptr()), ctx.handle, "async")
        ctx.synchronize()
        for j in range(len(wins)):
            n = int(totals[j].item())
            assert n == len(exp[j])
            got = bufs[j][: 2 * n].cpu().numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
            got = np.array(sorted(map(tuple, got.tolist())), np.int64).reshape(-1, 2)
            np.testing.assert_array_equal(got, exp[j])
        # capacity too small: the count still arrives
        po, pq = wins[0][0].c_struct(), wins[0][1].c_struct()
        _lib.check(L.gf_join_pp_async(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), r, 0,
                                      0, bufs[0].data_ptr(), 8, totals[0].data_ptr()), ctx.handle, "async small")
        ctx.synchronize()
        assert int(totals[0].item()) == len(exp[0])
    small = [(win(sf, wo_x, wo_y), win(sf, q_x, q_y)) for wo_x, wo_y, q_x, q_y in
             [(*oracle_mod.java_random_points(130, 3000, *BEIJING), *oracle_mod.java_random_points(131, 300, *BEIJING))]]
    exp0 = sf.PointPointJoinQuery(conf(sf), g, g).run(small[0][0], small[0][1], 0.0)
    buf = torch.zeros(2 * (len(exp0) + 16), dtype=torch.int32, device="cuda")
    po, pq = small[0][0].c_struct(), small[0][1].c_struct()
    torch.cuda.synchronize()
    _lib.check(L.gf_join_pp_async(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), 0.0, 0, 0,
                                  buf.data_ptr(), len(exp0) + 16, totals[1].data_ptr()), ctx.handle, "async r=0")
    ctx.synchronize()
    assert int(totals[1].item()) == len(exp0)


def test_join_dense_rows_fall_back_to_global(sf, oracle_mod):
    """A query row too dense to stage in LDS (every query point in one cell row) takes the
    task's global-memory probe; a single dense cell as well."""
    g = sf.UniformGrid(1000, *BEIJING)
    og = oracle_mod.grid(1000, *BEIJING)
    ox, oy = oracle_mod.java_random_points(91, 200_000, 115.5, 117.6, 40.0, 40.01)
    qx, qy = oracle_mod.java_random_points(92, 60_000, 115.5, 117.6, 40.002, 40.004)
    qx[:20_000] = 116.0 + 1e-7 * np.arange(20_000)
    st, pairs = oracle_mod.join_pp(og, og, ox, oy, qx, qy, 0.001)
    exp = np.array(sorted(map(tuple, pairs.tolist())), np.int64).reshape(-1, 2)
    got = sf.PointPointJoinQuery(conf(sf), g, g).run(win(sf, ox, oy), win(sf, qx, qy), 0.001)
    np.testing.assert_array_equal(got, exp)


def test_knn_hint_across_windows(sf, oracle_mod):
    """Continuous query: each window reuses the previous window's threshold hint.  A window
    whose neighbourhood was emptied (hint too small) must be re-evaluated, still exactly."""
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    N = 1_100_000
    for seed in (1, 2, 3, "hole", 4, "sparse", 5):
        if seed == "hole":  # nothing within 0.02 of the query: the carried hint finds < k points
            x, y = oracle_mod.java_random_points(99, N, *BEIJING)
            far = (x - QPOINT[0]) ** 2 + (y - QPOINT[1]) ** 2 > 0.02 ** 2
            x, y = x[far], y[far]
        elif seed == "sparse":  # fewer than k candidates within r at all
            x, y = oracle_mod.java_random_points(98, N, 117.3, 117.6, 40.8, 41.1)
            x[:20] = QPOINT[0] + np.linspace(0.01, 0.4, 20)
            y[:20] = QPOINT[1]
        else:
            x, y = oracle_mod.java_random_points(seed, N, *BEIJING)
        obj = np.random.default_rng(7).permutation(len(x)).astype(np.int64)
        res = op.run(win(sf, x, y, obj), q, 0.5, 50)
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, 50)
        check_knn(res, oo, od, oi)


def test_knn_pinned_records_async(sf, oracle_mod):
    """Several windows enqueued back to back with the record written by the kernel straight
    into mapped pinned host memory (no copy kernel), decoded after one sync."""
    import torch

    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    N, k = 1_200_000, 64
    wins, host = [], []
    for seed in (11, 12, 13):
        x, y = oracle_mod.java_random_points(seed, N, *BEIJING)
        obj = np.arange(N, dtype=np.int64) % 400_000  # duplicated objIDs: dedupe in select
        wins.append(win(sf, x, y, obj))
        host.append((x, y, obj))
    rec = sf.PinnedRecords(9, k)
    for i in range(9):
        op.enqueue(wins[i % 3], q, 0.5, k, rec.ptr(i))
    torch.cuda.synchronize()
    for i in range(9):
        x, y, obj = host[i % 3]
        res = op.finish(wins[i % 3], q, 0.5, k, rec.raw(i))
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
        check_knn(res, oo, od, oi)


@pytest.mark.parametrize("k,depth", [(50, 2), (120, 2), (50, 3), (120, 3), (50, 4), (120, 4), (300, 4)])
def test_knn_pipelined(sf, oracle_mod, k, depth):
    """Depth-2 pipeline: window i's select runs inside window i+1's fused scan kernel (depth 3:
    inside window i+2's, odd windows on a second stream); cold
    starts and a window whose carried hint is too small are re-evaluated at decode; the
    synchronous API on a pipelined plan."""
    import torch

    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    N = 1_100_000
    data = []
    for seed in (21, 22, "hole", 23, 24):
        if seed == "hole":
            x, y = oracle_mod.java_random_points(97, N, *BEIJING)
            far = (x - QPOINT[0]) ** 2 + (y - QPOINT[1]) ** 2 > 0.03 ** 2
            x, y = x[far], y[far]
        else:
            x, y = oracle_mod.java_random_points(seed, N, *BEIJING)
        obj = np.random.default_rng(3).permutation(len(x)).astype(np.int64)
        if seed == 23:  # trajectories: every objID three times
            obj %= len(x) // 3
        data.append((x, y, obj, win(sf, x, y, obj)))
    op.set_pipeline(0, q, 0.5, k, depth)
    order = [0, 1, 0, 1, 3, 4, 2, 3, 4, 0, 2, 2, 1]
    rec = sf.PinnedRecords(len(order), k)
    for i, j in enumerate(order):
        op.enqueue(data[j][3], q, 0.5, k, rec.ptr(i))
    op.flush(0, q, 0.5, k)
    torch.cuda.synchronize()
    for i, j in enumerate(order):
        x, y, obj, w = data[j]
        res = op.finish(w, q, 0.5, k, rec.raw(i))
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
        check_knn(res, oo, od, oi)
    for j in (2, 0, 4):  # synchronous API on a pipelined plan
        x, y, obj, w = data[j]
        res = op.run(w, q, 0.5, k)
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
        check_knn(res, oo, od, oi)
    for j0, j1 in ((0, 1), (3, 4), (1, 2)):  # windows built by torch right before the call
        (x0, y0, o0, w0), (x1, y1, o1, w1) = data[j0], data[j1]
        w = sf.PointWindow(torch.cat([w0.x, w1.x]), torch.cat([w0.y, w1.y]), torch.cat([w0.objID, w1.objID + 10**7]),
                           torch.cat([w0.timeStampMillisec, w1.timeStampMillisec]))
        res = op.run(w, q, 0.5, k)
        del w
        st, oo, od, oi = oracle_mod.knn(og, np.concatenate([x0, x1]), np.concatenate([y0, y1]),
                                        np.concatenate([o0, o1 + 10**7]), QPOINT[0], QPOINT[1], 0.5, k)
        check_knn(res, oo, od, oi)
    op.set_pipeline(0, q, 0.5, k, 1)


@pytest.mark.parametrize("layout", [0, 1])
def test_knn_merge_dev_batch(sf, oracle_mod, layout):
    """One batched merge launch over several windows' shard records (both layouts) == each
    window evaluated whole; shards use index bases so the merged idx is global."""
    import torch

    from spatialflink_amd import _lib

    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    k, S, W = 40, 3, 5
    rb = sf.spatialOperators.knn_record_bytes(k)
    recs = torch.zeros(S * W * rb, dtype=torch.uint8, device="cuda")
    expect = []
    ops = [sf.PointPointKNNQuery(conf(sf), g) for _ in range(S)]
    for wi in range(W):
        x, y = oracle_mod.java_random_points(300 + wi, 240_000, *BEIJING)
        obj = (np.random.default_rng(wi).permutation(len(x)) % 150_000).astype(np.int64)  # duplicates
        expect.append(oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k))
        for s, ix in enumerate(np.array_split(np.arange(len(x)), S)):
            ctx, plan = ops[s].plan(0, q, 0.5, k)
            _lib.check(_lib.lib().gf_knn_plan_set_index_base(plan, int(ix[0])), ctx.handle, "base")
            slot = s * W + wi if layout == 0 else wi * S + s
            ops[s].enqueue(win(sf, x[ix], y[ix], obj[ix]), q, 0.5, k, recs[slot * rb:(slot + 1) * rb])
    out = torch.zeros(W * rb, dtype=torch.uint8, device="cuda")
    ctx = _lib.context(0)
    _lib.check(_lib.lib().gf_knn_merge_dev_batch(ctx.handle, k, recs.data_ptr(), S, W, layout, out.data_ptr()),
               ctx.handle, "merge batch")
    raw = out.cpu().numpy().tobytes()
    for wi in range(W):
        st, o, d, i = sf.spatialOperators.decode_knn_record(raw[wi * rb:(wi + 1) * rb], k)
        est, eo, ed, ei = expect[wi]
        assert st == 0
        np.testing.assert_array_equal(o, eo)
        np.testing.assert_array_equal(d, ed)
        np.testing.assert_array_equal(i, ei)


def test_join_dense_spot_and_capacity(sf, oracle_mod):
    """Many pairs per point around a dense spot == the oracle; a too-small capacity returns
    GF_ERR_CAPACITY with the exact count."""
    import ctypes as C

    import torch

    from spatialflink_amd import _lib

    g = sf.UniformGrid(1000, *BEIJING)
    og = oracle_mod.grid(1000, *BEIJING)
    x, y = oracle_mod.java_random_points(71, 600_000, *BEIJING)
    qx, qy = oracle_mod.java_random_points(72, 60_000, *BEIJING)
    # a dense spot: many pairs per point (more than the LDS pair slots)
    qx[:2000] = 116.4 + 1e-5 * np.arange(2000) % 3e-4
    qy[:2000] = 40.0
    x[:3000] = 116.4001
    y[:3000] = 40.0
    st, exp = oracle_mod.join_pp(og, og, x, y, qx, qy, 0.001)
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    op = sf.PointPointJoinQuery(conf(sf), g)
    ctx = _lib.context(0)
    wo, wq = win(sf, x, y), win(sf, qx, qy)
    np.testing.assert_array_equal(op.run(wo, wq, 0.001), exp)
    pairs = torch.empty(2 * 100, dtype=torch.int32, device="cuda")
    n = C.c_int64()
    po, pq = wo.c_struct(), wq.c_struct()
    st = _lib.lib().gf_join_pp(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), 0.001, 0, 0,
                               pairs.data_ptr(), 100, C.byref(n))
    assert st == _lib.GF_ERR_CAPACITY and n.value == len(exp)
    # an output buffer that is only 4-byte aligned (two 4-byte stores per pair)
    big = torch.zeros(2 * len(exp) + 2, dtype=torch.int32, device="cuda")
    st = _lib.lib().gf_join_pp(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), 0.001, 0, 0,
                               big.data_ptr() + 4, len(exp), C.byref(n))
    assert st == 0 and n.value == len(exp)
    got = big[1:1 + 2 * len(exp)].cpu().numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
    np.testing.assert_array_equal(got[np.lexsort((got[:, 1], got[:, 0]))], exp)
    assert big[0].item() == 0 and big[-1].item() == 0  # nothing written outside the buffer


def test_join_band_global_window(sf, oracle_mod):
    """Band probe (the fine path) when even a one-sub-column window of a band cannot be staged:
    6000 query points inside one sub-cell (120 KB of staging against the ~86 KB budget) -- that
    sub-column's candidates are read from global memory, the rest of the band from windows in LDS
    -- plus a second dense spot that needs several windows; == the oracle, then the same window
    again (regions sized from the first call's per-block counts)."""
    g = sf.UniformGrid(1000, *BEIJING)
    og = oracle_mod.grid(1000, *BEIJING)
    x, y = oracle_mod.java_random_points(91, 300_000, *BEIJING)
    qx, qy = oracle_mod.java_random_points(92, 50_000, *BEIJING)
    rng = np.random.default_rng(93)
    qx[:6000] = 116.4 + rng.uniform(0.0, 2e-4, 6000)      # one sub-cell (side 0.00105)
    qy[:6000] = 40.0 + rng.uniform(0.0, 2e-4, 6000)
    qx[6000:12000] = 116.1 + rng.uniform(0.0, 0.02, 6000)  # a dense stretch of one row band
    qy[6000:12000] = 40.3 + rng.uniform(0.0, 2e-3, 6000)
    x[:1500] = 116.4 + rng.uniform(-1e-3, 1.2e-3, 1500)
    y[:1500] = 40.0 + rng.uniform(-1e-3, 1.2e-3, 1500)
    x[1500:4000] = 116.1 + rng.uniform(0.0, 0.02, 2500)
    y[1500:4000] = 40.3 + rng.uniform(0.0, 2e-3, 2500)
    st, exp = oracle_mod.join_pp(og, og, x, y, qx, qy, 0.001)
    assert st == 0 and len(exp) > 1_000_000
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    op = sf.PointPointJoinQuery(conf(sf), g)
    wo, wq = win(sf, x, y), win(sf, qx, qy)
    for _ in range(2):
        np.testing.assert_array_equal(op.run(wo, wq, 0.001), exp)


# ------------------------------------------------------------------ point-polygon join
def test_join_ppoly_golden(sf):
    f = load("join_ppoly.npz")
    g = sf.UniformGrid(100, *BEIJING)
    polys = golden_polygons(sf, f, g)
    w = win(sf, f["x"], f["y"])
    for r in (0.001, 0.05, 0.3, 0.0):
        for ap in (0, 1):
            got = sf.PointPolygonJoinQuery(conf(sf, bool(ap)), g, g).run(w, polys, r)
            np.testing.assert_array_equal(got, f[f"r{r}_a{ap}"], err_msg=f"r={r} ap={ap}")


@pytest.mark.parametrize("n,r,metric", [(500, 0.001, 0), (100, 0.05, 0), (500, 0.01, 1), (1000, 0.004, 0)])
def test_join_ppoly_generated_1000(sf, oracle_mod, n, r, metric):
    """C3's 1000 query polygons as the polygon side of the join, test-sized point window."""
    g = sf.UniformGrid(n, *BEIJING)
    og = oracle_mod.grid(n, *BEIJING)
    raw = oracle_mod.generate_query_polygons(1000, 115.5, 39.6, 117.6, 41.1)
    polys = [sf.Polygon(p, g) for p in raw]
    x, y = oracle_mod.java_random_points(33, 200_000, 115.45, 115.75, *BEIJING[2:])
    w = win(sf, x, y)
    for ap in (False, True):
        got = sf.PointPolygonJoinQuery(conf(sf, ap, metric), g, g).run(w, polys, r)
        exp = oracle_mod.join_ppoly(og, og, x, y, oracle_mod.Polygons(raw), r, ap, metric)
        exp = np.array(sorted(map(tuple, exp.tolist())), np.int64).reshape(-1, 2)
        assert len(exp) > 0
        np.testing.assert_array_equal(got, exp, err_msg=f"approximate={ap}")


def test_join_ppoly_capacity_empty_and_grid_mismatch(sf, oracle_mod):
    import ctypes as C

    import torch
    from spatialflink_amd import _lib

    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    raw = oracle_mod.generate_query_polygons(100, 115.5, 39.6, 117.6, 41.1)
    polys = [sf.Polygon(p, g) for p in raw]
    x, y = oracle_mod.java_random_points(35, 50_000, *BEIJING)
    w = win(sf, x, y)
    exp = oracle_mod.join_ppoly(og, og, x, y, oracle_mod.Polygons(raw), 0.05)
    ctx = _lib.context(0)
    L = _lib.lib()
    ps = sf.PolygonSet(polys)
    cs = ps.c_struct()
    h = C.c_void_p()
    _lib.check(L.gf_join_ppoly_plan_create(ctx.handle, C.byref(g.c_grid), C.byref(cs), 0.05, 0, 0, C.byref(h)),
               ctx.handle, "plan")
    try:
        pts = w.c_struct()
        npairs = C.c_int64()
        # counting call (no buffer), then a too-small buffer, then the right size
        assert L.gf_join_ppoly_run(h, C.byref(g.c_grid), C.byref(pts), None, 0, C.byref(npairs)) == _lib.GF_ERR_CAPACITY
        assert npairs.value == len(exp)
        small = torch.empty(2 * 10, dtype=torch.int32, device="cuda")
        assert L.gf_join_ppoly_run(h, C.byref(g.c_grid), C.byref(pts), small.data_ptr(), 10,
                                   C.byref(npairs)) == _lib.GF_ERR_CAPACITY
        assert npairs.value == len(exp)
        full = torch.empty(2 * len(exp), dtype=torch.int32, device="cuda")
        assert L.gf_join_ppoly_run(h, C.byref(g.c_grid), C.byref(pts), full.data_ptr(), len(exp), C.byref(npairs)) == 0
        got = full.cpu().numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
        assert sorted(map(tuple, got.tolist())) == sorted(map(tuple, exp.tolist()))
        # empty window
        e = win(sf, np.zeros(0), np.zeros(0)).c_struct()
        assert L.gf_join_ppoly_run(h, C.byref(g.c_grid), C.byref(e), full.data_ptr(), 4, C.byref(npairs)) == 0
        assert npairs.value == 0
        # the point grid must equal the polygon grid; a range plan is not a join plan
        g2 = sf.UniformGrid(101, *BEIJING)
        assert L.gf_join_ppoly_run(h, C.byref(g2.c_grid), C.byref(pts), full.data_ptr(), 4,
                                   C.byref(npairs)) == _lib.GF_ERR_ARG
    finally:
        L.gf_range_plan_destroy(h)
    # the one-shot entry point
    npairs = C.c_int64()
    full = torch.empty(2 * len(exp), dtype=torch.int32, device="cuda")
    pts = w.c_struct()
    assert L.gf_join_ppoly(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(pts), C.byref(cs), 0.05, 0, 0,
                           full.data_ptr(), len(exp), C.byref(npairs)) == 0
    assert npairs.value == len(exp)


def test_join_ppoly_dense_overlap_worklist_overflow(sf, oracle_mod):
    """60 overlapping triangles (not rectangles: every pair needs the exact JTS distance) over
    the same spot: a block round's exact-distance worklist overflows and points are recounted
    by their own walk; plus a polygon with a hole."""
    g = sf.UniformGrid(200, *BEIJING)
    og = oracle_mod.grid(200, *BEIJING)
    raw = []
    for k in range(60):
        d = 0.0004 * k
        raw.append([[(116.0 + d, 40.0), (116.08 + d, 40.01), (116.03, 40.07 + d), (116.0 + d, 40.0)]])
    raw.append([[(116.0, 39.98), (116.12, 39.98), (116.12, 40.1), (116.0, 40.1), (116.0, 39.98)],
                [(116.02, 40.0), (116.05, 40.0), (116.05, 40.03), (116.02, 40.03), (116.02, 40.0)]])
    polys = [sf.Polygon(p, g) for p in raw]
    x, y = oracle_mod.java_random_points(37, 60_000, 115.98, 116.15, 39.97, 40.12)
    w = win(sf, x, y)
    for r in (0.002, 0.02):
        got = sf.PointPolygonJoinQuery(conf(sf), g, g).run(w, polys, r)
        exp = oracle_mod.join_ppoly(og, og, x, y, oracle_mod.Polygons(raw), r)
        exp = np.array(sorted(map(tuple, exp.tolist())), np.int64).reshape(-1, 2)
        assert len(exp) > 100_000
        np.testing.assert_array_equal(got, exp, err_msg=f"r={r}")


def test_range_windows_in_flight_on_two_contexts(sf, oracle_mod):
    """Consecutive windows alternating over two contexts (two HIP streams, two plans), as the
    bench's --range-streams 2 runs them: every window's hits == the oracle's."""
    import ctypes as C

    import torch
    from spatialflink_amd import _lib

    L = _lib.lib()
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    qx, qy = np.array([QPOINT[0]]), np.array([QPOINT[1]])
    ctxs = [_lib.Context(0), _lib.Context(0)]
    plans = []
    for c in ctxs:
        h = C.c_void_p()
        _lib.check(L.gf_range_pp_plan_create(c.handle, C.byref(g.c_grid), qx.ctypes.data, qy.ctypes.data, 1, 0.3, 0, 0,
                                             C.byref(h)), c.handle, "plan")
        plans.append(h)
    try:
        wins, exps = [], []
        for j in range(6):
            x, y = oracle_mod.java_random_points(70 + j, 300_000, *BEIJING)
            wins.append(win(sf, x, y))
            exps.append(oracle_mod.range_pp(og, x, y, qx, qy, 0.3))
        torch.cuda.synchronize()
        n = 300_000
        bitmaps = torch.zeros(6, (n + 63) // 64, dtype=torch.int64, device="cuda")
        counts = torch.zeros(6, 2, dtype=torch.int64, device="cuda")
        # the raw contexts run on their own non-blocking streams: order them after torch's fills
        torch.cuda.synchronize()
        pts = [w.c_struct() for w in wins]
        for j in range(6):
            _lib.check(L.gf_range_run(plans[j % 2], C.byref(pts[j]), bitmaps[j].data_ptr(), None, counts[j].data_ptr()),
                       ctxs[j % 2].handle, "gf_range_run")
        for c in ctxs:
            c.synchronize()
        for j in range(6):
            got = sf.spatialOperators.bitmap_indices(ctxs[0], bitmaps[j], n).astype(np.int64)
            np.testing.assert_array_equal(got, exps[j], err_msg=f"window {j}")
            assert int(counts[j, 0].item()) == len(exps[j])
    finally:
        for h in plans:
            L.gf_range_plan_destroy(h)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1_000_000, 10_000_001, 40_000_003])
def test_bitmap_to_indices_async(sf, n):
    """One-launch async expansion == the synchronous one (ascending indices, count on the
    device, indices past cap not written, bits past n ignored), on random bitmaps of every
    density; 40M points = 1221 blocks, so the look-back walks more than one 512-block round."""
    import ctypes as C

    import torch
    from spatialflink_amd import _lib

    ctx = _lib.context(0)
    L = _lib.lib()
    rng = np.random.default_rng(n)
    words = (n + 63) // 64
    for dens in (0.0, 0.01, 0.5, 1.0):
        bits = rng.random(words * 64) < dens
        bits[n:] = dens == 1.0  # the last word's bits past n are ignored
        bm = torch.from_numpy(np.packbits(bits.reshape(-1, 8)[:, ::-1]).view(np.int64).copy()).cuda()
        exp = np.flatnonzero(bits[:n])
        for cap in (len(exp), max(len(exp) // 2, 0)):
            idx = torch.full((max(cap, 1),), -1, dtype=torch.int32, device="cuda")
            cnt = torch.full((1,), -7, dtype=torch.int64, device="cuda")
            _lib.check(L.gf_bitmap_to_indices_async(ctx.handle, bm.data_ptr(), n, idx.data_ptr(), cap, cnt.data_ptr()),
                       ctx.handle, "async")
            assert int(cnt.item()) == len(exp)
            got = idx.cpu().numpy().view(np.uint32).astype(np.int64)[:cap]
            np.testing.assert_array_equal(got, exp[:cap])


def test_range_counts_folded_in_kernel(sf, oracle_mod):
    """The window's counts come from the last block of the window's last kernel (ticket):
    consecutive windows on one plan, inline and deferred candidate tests, every count right."""
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    raw = oracle_mod.generate_query_polygons(200, BEIJING[0], BEIJING[2], BEIJING[1], BEIJING[3])
    polys = [sf.Polygon(rings, g) for rings in raw]
    op = sf.PointPolygonRangeQuery(conf(sf), g)
    qop = sf.PointPointRangeQuery(conf(sf), g)
    q = sf.Point("q", *QPOINT, 0, g)
    for j in range(5):
        x, y = oracle_mod.java_random_points(500 + j, 400_000 + 77 * j, *BEIJING)
        w = win(sf, x, y)
        res = op.run(w, polys, 0.002)
        assert res.count() == len(oracle_mod.range_ppoly(og, x, y, oracle_mod.Polygons(raw), 0.002))
        res = qop.run(w, [q], 0.3)
        assert res.count() == len(oracle_mod.range_pp(og, x, y, [QPOINT[0]], [QPOINT[1]], 0.3))


@pytest.mark.parametrize("kind", ["arith", "table", "poly"])
def test_range_run_batch(sf, oracle_mod, kind):
    """gf_range_run_batch: up to 16 windows of one plan in one launch (+ one index-list launch),
    windows of every size (0, 1, ragged, 1M) -- each window's counts, bitmap and index list equal
    the oracle's over that window alone."""
    import ctypes as C

    import torch
    from spatialflink_amd import _lib

    L = _lib.lib()
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    ctx = _lib.context(0)
    h = C.c_void_p()
    if kind == "poly":
        raw = oracle_mod.generate_query_polygons(50, 115.5, 39.6, 117.6, 41.1)
        ps = sf.PolygonSet([sf.Polygon(p, g) for p in raw])
        cs = ps.c_struct()
        _lib.check(L.gf_range_ppoly_plan_create(ctx.handle, C.byref(g.c_grid), C.byref(cs), 0.01, 0, 0, C.byref(h)),
                   ctx.handle, "plan")
        expect = lambda x, y: oracle_mod.range_ppoly(og, x, y, oracle_mod.Polygons(raw), 0.01)  # noqa: E731
    else:
        qx = np.array([QPOINT[0]] + ([116.9, 117.2] if kind == "table" else []))
        qy = np.array([QPOINT[1]] + ([40.3, 40.8] if kind == "table" else []))
        r = 0.5 if kind == "arith" else 0.03
        _lib.check(L.gf_range_pp_plan_create(ctx.handle, C.byref(g.c_grid), qx.ctypes.data, qy.ctypes.data, len(qx),
                                             r, 0, 0, C.byref(h)), ctx.handle, "plan")
        expect = lambda x, y: oracle_mod.range_pp(og, x, y, qx, qy, r)  # noqa: E731
    try:
        sizes = [1_000_000, 0, 1, 63, 64, 65, 70_001, 1_000_000, 333_333, 5, 2]
        wins = []
        for j, n in enumerate(sizes):
            x, y = oracle_mod.java_random_points(500 + j, n, 115.4, 117.7, 39.5, 41.2)
            wins.append((x, y, win(sf, x, y)))
        B = len(sizes)
        pts = (_lib.GfPoints * B)(*[w[2].c_struct() for w in wins])
        bms = [torch.zeros(max(1, (n + 63) // 64), dtype=torch.int64, device="cuda") for n in sizes]
        cnts = [torch.full((2,), -1, dtype=torch.int64, device="cuda") for _ in sizes]
        idxs = [torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda") for n in sizes]
        icnt = [torch.full((1,), -1, dtype=torch.int64, device="cuda") for _ in sizes]
        P_ = C.c_void_p
        for rep in range(2):  # the second call reuses the tickets / partials the first reset
            st = L.gf_range_run_batch(h, B, pts, (P_ * B)(*[b.data_ptr() for b in bms]),
                                      (P_ * B)(*[c.data_ptr() for c in cnts]),
                                      (P_ * B)(*[i.data_ptr() for i in idxs]), (C.c_int64 * B)(*sizes),
                                      (P_ * B)(*[c.data_ptr() for c in icnt]))
            _lib.check(st, ctx.handle, "gf_range_run_batch")
            torch.cuda.synchronize()
            for j, (x, y, w) in enumerate(wins):
                exp = expect(x, y)
                assert int(cnts[j][0]) == len(exp) == int(icnt[j][0]), (kind, j)
                np.testing.assert_array_equal(idxs[j][:len(exp)].cpu().numpy().astype(np.int64), exp)
                got = sf.spatialOperators.bitmap_indices(ctx, bms[j], sizes[j]).astype(np.int64)
                np.testing.assert_array_equal(got, exp)
    finally:
        L.gf_range_plan_destroy(h)


@pytest.mark.parametrize("depth", [3, 4])
def test_knn_enqueue_fresh_torch_windows(sf, oracle_mod, depth):
    """Windows produced by torch on the context stream right before an ASYNC depth >= 3 enqueue
    (windows launch on the plan's other streams, which do not wait for the context
    stream): PointPointKNNQuery.enqueue orders them after the window's first use, so every
    record == the oracle's."""
    import torch

    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    k, N = 50, 1_100_000
    base = []
    for seed in (61, 62, 63):
        x, y = oracle_mod.java_random_points(seed, N, *BEIJING)
        base.append((x, y, np.arange(N, dtype=np.int64) + seed * 10_000_000))
    dev = [sf.PointWindow.from_numpy(*b) for b in base]
    op.set_pipeline(0, q, 0.5, k, depth)
    order = [(0, 1), (1, 2), (2, 0), (0, 2), (1, 0), (2, 1)]
    rec = sf.PinnedRecords(len(order), k)
    expect = []
    keep = []  # a window's memory must stay valid until its record is complete (the C ABI's rule)
    for i, (a, b) in enumerate(order):
        # a fresh window: torch kernels on the current stream write it just before the enqueue
        w = sf.PointWindow(torch.cat([dev[a].x, dev[b].x]) * 1.0, torch.cat([dev[a].y, dev[b].y]) * 1.0,
                           torch.cat([dev[a].objID, dev[b].objID]), torch.cat([dev[a].timeStampMillisec,
                                                                                dev[b].timeStampMillisec]))
        op.enqueue(w, q, 0.5, k, rec.ptr(i))
        expect.append(oracle_mod.knn(og, np.concatenate([base[a][0], base[b][0]]), np.concatenate([base[a][1], base[b][1]]),
                                     np.concatenate([base[a][2], base[b][2]]), QPOINT[0], QPOINT[1], 0.5, k))
        keep.append(w)
    op.flush(0, q, 0.5, k)
    torch.cuda.synchronize()
    for i in range(len(order)):
        st, o, d, ix = rec.decode(i)
        est, eo, ed, ei = expect[i]
        assert st == 0
        np.testing.assert_array_equal(o, eo)
        np.testing.assert_array_equal(d, ed)
        np.testing.assert_array_equal(ix, ei)
    op.set_pipeline(0, q, 0.5, k, 1)
