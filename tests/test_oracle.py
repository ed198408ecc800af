"""CPU: the oracle (C restatement) against the committed golden fixtures and the
independent Python restatement.  Parity with the reference is unpinned (no reference
fixtures exist); these tests pin the oracle to its own cross-checked fixtures and to the
reference facts that can be derived by reading the Java."""
import os

import numpy as np
import pytest

from conftest import BEIJING, GOLDEN, QPOINT


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def test_grid_constants(oracle_mod):
    O = oracle_mod
    # UniformGrid(int, ...) does not square the bounds: (117.6-115.5)/n in binary64
    assert O.grid(100, *BEIJING).cellLength == 0.020999999999999942
    assert O.grid(500, *BEIJING).cellLength == 0.0041999999999999885
    assert O.grid(1000, *BEIJING).cellLength == 0.0020999999999999942


def test_java_random(oracle_mod):
    x, y = oracle_mod.java_random_points(42, 2, 0.0, 1.0, 0.0, 1.0)
    # new java.util.Random(42).nextDouble() sequence
    assert x[0] == 0.7275636800328681 and y[0] == 0.6832234717598454


def test_cell_id_format_parse(oracle_mod):
    O = oracle_mod
    assert O.cell_id(3, 45) == "0000300045"
    assert O.cell_id(-1, 5) == "-000100005"   # String.format("%05d", -1)
    assert O.parse_cell_id("-000100005") == (-1, 5)
    assert O.parse_cell_id("0000000000") == (0, 0)
    assert O.parse_cell_id("9999999999") == (99999, 99999)


def test_jint(oracle_mod):
    O = oracle_mod
    assert O.jint(float("nan")) == 0
    assert O.jint(1e300) == 2147483647 and O.jint(-1e300) == -2147483648
    assert O.jint(-0.5) == 0 and O.jint(2.9) == 2


def test_layers(oracle_mod):
    g = oracle_mod.grid(100, *BEIJING)
    assert oracle_mod.layers(g, 0.5) == (15, 24)
    assert oracle_mod.layers(g, 0.05) == (0, 3)
    assert oracle_mod.layers(g, 0.02) == (-1, 1)
    assert oracle_mod.layers(g, 0.0) == (-1, 0)


def test_gc_set_sizes(oracle_mod):
    g = oracle_mod.grid(100, *BEIJING)
    qcx, qcy = oracle_mod.assign_cells(g, [QPOINT[0]], [QPOINT[1]])
    gs, cs = oracle_mod.gc_sets_point(g, 0.5, qcx[0], qcy[0])
    assert len(gs) == 31 * 31 and not (gs & cs)
    # g == 0: the query cell itself, no validKey (UniformGrid.java:171-174)
    gs0, _ = oracle_mod.gc_sets_point(g, 0.05, -3, 7)
    assert gs0 == {(-3, 7)}


def test_generate_query_polygons(oracle_mod):
    polys = oracle_mod.generate_query_polygons(1000, 115.5, 39.6, 117.6, 41.1)
    assert len(polys) == 1000  # 10 columns x 100 squares of side 0.015
    ring = polys[0][0]
    assert ring[0] == ring[-1] and len(ring) == 5
    assert abs((ring[1][0] - ring[0][0]) - 0.015) < 1e-15


@pytest.mark.parametrize("n", [100, 500])
def test_cells_golden(oracle_mod, n):
    f = load(f"cells_n{n}.npz")
    g = oracle_mod.grid(n, *BEIJING)
    cx, cy = oracle_mod.assign_cells(g, f["x"], f["y"])
    np.testing.assert_array_equal(cx, f["cx"])
    np.testing.assert_array_equal(cy, f["cy"])


def test_range_pp_golden(oracle_mod):
    f = load("range_pp.npz")
    g = oracle_mod.grid(100, *BEIJING)
    for qn in ("q1", "q3"):
        for r in (0.5, 0.05, 0.02, 0.0):
            for ap in (0, 1):
                got = oracle_mod.range_pp(g, f["x"], f["y"], f[f"{qn}_qx"], f[f"{qn}_qy"], r, bool(ap))
                np.testing.assert_array_equal(got, f[f"{qn}_r{r}_a{ap}"])


def test_range_ppoly_golden(oracle_mod):
    f = load("range_ppoly.npz")
    g = oracle_mod.grid(100, *BEIJING)
    P = oracle_mod.Polygons([])
    P.ring_off, P.vert_off, P.vx, P.vy = f["ring_off"], f["vert_off"], f["vx"], f["vy"]
    P.c = oracle_mod.OrcPolygons(len(P.ring_off) - 1, P.ring_off.ctypes.data, P.vert_off.ctypes.data,
                                 P.vx.ctypes.data, P.vy.ctypes.data)
    for r in (0.001, 0.05, 0.3):
        for ap in (0, 1):
            got = oracle_mod.range_ppoly(g, f["x"], f["y"], P, r, bool(ap))
            np.testing.assert_array_equal(got, f[f"r{r}_a{ap}"])


def test_knn_golden(oracle_mod):
    f = load("knn.npz")
    g = oracle_mod.grid(100, *BEIJING)
    for r in (0.5, 0.05, 0.3):
        for k in (1, 50, 100):
            for tag, ob in (("u", f["objID"]), ("d", f["objID_dup"])):
                st, oo, od, oi = oracle_mod.knn(g, f["x"], f["y"], ob, QPOINT[0], QPOINT[1], r, k)
                assert st == 0
                np.testing.assert_array_equal(oo, f[f"{tag}_r{r}_k{k}_obj"])
                np.testing.assert_array_equal(od, f[f"{tag}_r{r}_k{k}_d"])
                np.testing.assert_array_equal(oi, f[f"{tag}_r{r}_k{k}_idx"])


def test_knn_reference_shaped_agrees_on_unique_ids(oracle_mod):
    """With unique objIDs and distinct distances the Java-shaped evaluator (per-cell
    PriorityQueues + windowAll merge, bug included) returns the contract's set."""
    f = load("knn.npz")
    g = oracle_mod.grid(100, *BEIJING)
    for r in (0.5, 0.05):
        st, oo, od, oi = oracle_mod.knn(g, f["x"], f["y"], f["objID"], QPOINT[0], QPOINT[1], r, 50,
                                        reference_shaped=True)
        assert st == 0
        ref = sorted(zip(od.tolist(), oo.tolist()))
        assert ref == list(zip(f[f"u_r{r}_k50_d"].tolist(), f[f"u_r{r}_k50_obj"].tolist()))


def test_knn_reference_k1_npe(oracle_mod):
    """k == 1 throws a NullPointerException in KNNQuery.java:249-251 on the first eviction."""
    f = load("knn.npz")
    g = oracle_mod.grid(100, *BEIJING)
    st, *_ = oracle_mod.knn(g, f["x"], f["y"], f["objID"], QPOINT[0], QPOINT[1], 0.5, 1, reference_shaped=True)
    assert st == oracle_mod.ERR_NPE


def test_join_golden(oracle_mod):
    f = load("join.npz")
    g = oracle_mod.grid(100, *BEIJING)
    for r in (0.001, 0.05, 0.0):
        for ap in (0, 1):
            if r == 0.0 and ap:
                continue
            st, pairs = oracle_mod.join_pp(g, g, f["ox"], f["oy"], f["qx"], f["qy"], r, bool(ap))
            assert st == 0
            got = np.array(sorted(map(tuple, pairs.tolist())), np.int64).reshape(-1, 2)
            np.testing.assert_array_equal(got, f[f"r{r}_a{ap}"])


def test_join_negative_radius_exits(oracle_mod):
    g = oracle_mod.grid(100, *BEIJING)
    st, _ = oracle_mod.join_pp(g, g, [116.0], [40.0], [116.0], [40.0], -0.1)
    assert st == oracle_mod.ERR_LAYERS


def test_oracle_vs_pyref_random(oracle_mod):
    import pyref as P

    g = oracle_mod.grid(37, *BEIJING)
    pg = P.Grid(37, *BEIJING)
    x, y = oracle_mod.java_random_points(5, 1500, *BEIJING)
    for r in (0.2, 0.07):
        a = oracle_mod.range_pp(g, x, y, [QPOINT[0]], [QPOINT[1]], r)
        assert a.tolist() == P.range_pp(pg, x.tolist(), y.tolist(), [QPOINT], r)


def test_hypot_basics(oracle_mod):
    O = oracle_mod
    assert O.hypot(3.0, 4.0) == 5.0
    assert O.hypot(0.0, 0.0) == 0.0
    assert O.hypot(float("inf"), float("nan")) == float("inf")
    assert abs(O.hypot(1e308, 1e308) / np.hypot(1e308, 1e308) - 1) < 1e-15
    assert O.hypot(1e-310, 3e-310) == np.hypot(1e-310, 3e-310) or abs(O.hypot(1e-310, 3e-310) - np.hypot(1e-310, 3e-310)) <= 5e-324
    x = np.random.default_rng(1).uniform(-1, 1, (2000, 2))
    for a, b in x:
        assert abs(O.hypot(a, b) - np.hypot(a, b)) <= 2 * np.spacing(np.hypot(a, b))


def _fixture_polygons(oracle_mod, f):
    P = oracle_mod.Polygons([])
    P.ring_off, P.vert_off, P.vx, P.vy = f["ring_off"], f["vert_off"], f["vx"], f["vy"]
    P.c = oracle_mod.OrcPolygons(len(P.ring_off) - 1, P.ring_off.ctypes.data, P.vert_off.ctypes.data,
                                 P.vx.ctypes.data, P.vy.ctypes.data)
    return P


def test_join_ppoly_golden(oracle_mod):
    """PointPolygonJoinQuery (JoinQuery.java:93-115, PointPolygonJoinQuery.java:154-213): the
    fixture was cross-checked against tests/golden/pyref.py when written."""
    f = load("join_ppoly.npz")
    g = oracle_mod.grid(100, *BEIJING)
    P = _fixture_polygons(oracle_mod, f)
    for r in (0.001, 0.05, 0.3, 0.0):
        for ap in (0, 1):
            got = oracle_mod.join_ppoly(g, g, f["x"], f["y"], P, r, bool(ap))
            got = np.array(sorted(map(tuple, got.tolist())), np.int64).reshape(-1, 2)
            np.testing.assert_array_equal(got, f[f"r{r}_a{ap}"], err_msg=f"r={r} ap={ap}")


def test_join_ppoly_own_guaranteed_set(oracle_mod):
    """A polygon's candidate keys exclude only its OWN guaranteed cells (the replicated stream
    is per polygon), unlike the range query's global G: with two overlapping polygons every
    key of each is replicated, so a point in a cell guaranteed for one polygon still pairs with
    the other when within r."""
    import pyref as PR

    g = oracle_mod.grid(50, *BEIJING)
    pg = PR.Grid(50, *BEIJING)
    polys = [[[(116.0, 40.0), (116.2, 40.0), (116.2, 40.2), (116.0, 40.2), (116.0, 40.0)]],
             [[(116.25, 40.0), (116.4, 40.0), (116.4, 40.2), (116.25, 40.0)]]]
    x, y = oracle_mod.java_random_points(9, 3000, 115.9, 116.5, 39.9, 40.3)
    for r in (0.05, 0.13):
        got = sorted(map(tuple, oracle_mod.join_ppoly(g, g, x, y, oracle_mod.Polygons(polys), r).tolist()))
        assert got == PR.join_ppoly(pg, pg, x.tolist(), y.tolist(), polys, r)
        assert {q for _, q in got} == {0, 1}


@pytest.mark.parametrize("r,k,dup", [(0.5, 50, False), (0.05, 20, True), (0.3, 300, True), (0.5, 1, False),
                                     (0.002, 50, False)])
def test_cpu_baselines_match(oracle_mod, r, k, dup):
    """The bench's multi-core CPU baselines compute the same results as the single-thread
    oracle: the Flink-shaped parallel evaluator == the reference-shaped one (per-cell heaps +
    windowAll merge, bug included), the OpenMP scan == the build contract."""
    og = oracle_mod.grid(500, *BEIJING)
    x, y = oracle_mod.java_random_points(17, 200_000, 115.4, 117.7, 39.5, 41.2)
    obj = ((np.arange(len(x)) * 7919) % (60_000 if dup else len(x))).astype(np.int64)
    ref = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k, reference_shaped=True)
    con = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
    for T in (1, 3, 8):
        mt = oracle_mod.knn_mt(og, x, y, obj, QPOINT[0], QPOINT[1], r, k, T)
        assert mt[0] == ref[0]
        if ref[0] == 0:
            for a, b in zip(mt[1:], ref[1:]):
                np.testing.assert_array_equal(a, b)
        om = oracle_mod.knn_mt(og, x, y, obj, QPOINT[0], QPOINT[1], r, k, T, optimized=True)
        for a, b in zip(om, con):
            np.testing.assert_array_equal(a, b)


def test_synthetic_clustered_deterministic_and_in_bounds():
    import spatialflink_amd as sf

    a = sf.synthetic_clustered(3, 50_000, *BEIJING, centers=[QPOINT])
    b = sf.synthetic_clustered(3, 50_000, *BEIJING, centers=[QPOINT])
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    x, y = a
    assert (x >= BEIJING[0]).all() and (x < BEIJING[1]).all() and (y >= BEIJING[2]).all() and (y < BEIJING[3]).all()
    # 80% in 8 spots of sigma 0.01: the spot on the query point holds ~10% within 3 sigma
    near = np.hypot(x - QPOINT[0], y - QPOINT[1]) < 0.03
    assert 0.08 < near.mean() < 0.12


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_multicore_baselines_equal_serial(oracle_mod, threads):
    """The bench's multi-core CPU baseline lines (reference-shaped with Flink parallelism, and
    the optimised OpenMP scans) return exactly the serial restatements' results."""
    O = oracle_mod
    B = (115.5, 117.6, 39.6, 41.1)
    x, y = O.java_random_points(3, 60_000, 115.4, 117.7, 39.5, 41.2)
    x[:5] = np.nan
    for n, qs, r in ((100, [(116.414899, 39.920374)], 0.5), (100, [(116.4, 40.0), (117.0, 40.5), (115.3, 39.5)], 0.05),
                     (500, [(116.414899, 39.920374)], 0.002)):
        g = O.grid(n, *B)
        qx, qy = [q[0] for q in qs], [q[1] for q in qs]
        for ap in (False, True):
            exp = O.range_pp(g, x, y, qx, qy, r, ap)
            assert np.array_equal(O.range_pp_mt(g, x, y, qx, qy, r, threads, ap), exp)
            assert np.array_equal(O.range_pp_mt(g, x, y, qx, qy, r, threads, ap, optimized=True), exp)
    g = O.grid(500, *B)
    polys = O.Polygons(O.generate_query_polygons(1000, 115.5, 39.6, 117.6, 41.1))
    xs, ys = O.java_random_points(4, 40_000, 115.45, 115.75, *B[2:])
    for r, ap in ((0.001, False), (0.001, True), (0.05, False)):
        exp = O.range_ppoly(g, xs, ys, polys, r, ap)
        assert np.array_equal(O.range_ppoly_mt(g, xs, ys, polys, r, threads, ap), exp)
        assert np.array_equal(O.range_ppoly_mt(g, xs, ys, polys, r, threads, ap, optimized=True), exp)
    g = O.grid(1000, *B)
    qx, qy = O.java_random_points(5, 8_000, 115.4, 117.7, 39.5, 41.2)
    for r in (0.001, 0.004):
        st, exp = O.join_pp(g, g, x, y, qx, qy, r)
        exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
        assert np.array_equal(O.join_pp_mt(g, g, x, y, qx, qy, r, threads), exp)
        assert np.array_equal(O.join_pp_mt(g, g, x, y, qx, qy, r, threads, optimized=True), exp)
    text = b"".join(b"%d,%d,%.9f,%.9f\n" % (i, 1000 + i, 116 + i * 1e-6, 40 - i * 1e-6) for i in range(5000))
    ex, ey, eo, et, bl, bk = O.csv_parse(text, ",", (0, 1, 2, 3))
    mx, my, mt, mbl, mbk = O.csv_parse_mt(text, ",", (0, 1, 2, 3), threads)
    assert bl == mbl == -1 and np.array_equal(ex, mx) and np.array_equal(ey, my) and np.array_equal(et, mt)


def test_join_ppoly_mt_matches_serial(oracle_mod):
    """The point-polygon join's CPU baseline with Flink parallelism T (orc_join_ppoly_mt) returns
    the serial restatement's pair set."""
    import numpy as np

    g = oracle_mod.grid(500, 115.5, 117.6, 39.6, 41.1)
    x, y = oracle_mod.java_random_points(5, 100_000, 115.5, 117.6, 39.6, 41.1)
    P = oracle_mod.Polygons(oracle_mod.generate_query_polygons(1000, 115.5, 39.6, 117.6, 41.1))
    a = oracle_mod.join_ppoly(g, g, x, y, P, 0.001)
    a = a[np.lexsort((a[:, 1], a[:, 0]))]
    for T in (1, 3, 8):
        assert np.array_equal(oracle_mod.join_ppoly_mt(g, g, x, y, P, 0.001, T), a)


def test_knn_ppoly_mt_matches_serial(oracle_mod):
    """Polygon kNN's CPU baseline with Flink parallelism T (orc_knn_ppoly_mt) == the serial contract."""
    import numpy as np

    g = oracle_mod.grid(500, 115.5, 117.6, 39.6, 41.1)
    x, y = oracle_mod.java_random_points(6, 200_000, 115.5, 117.6, 39.6, 41.1)
    obj = np.arange(len(x), dtype=np.int64) % 150_000  # duplicated objIDs: the dedupe matters
    sq = [[(116.40, 39.91), (116.42, 39.91), (116.42, 39.93), (116.40, 39.93), (116.40, 39.91)]]
    P = oracle_mod.Polygons([sq])
    ref = oracle_mod.knn_ppoly(g, x, y, obj, P, 0.5, 50)
    for T in (1, 4, 7):
        got = oracle_mod.knn_ppoly_mt(g, x, y, obj, P, 0.5, 50, T)
        assert got[0] == ref[0] and all(np.array_equal(a, b) for a, b in zip(got[1:], ref[1:]))


def test_join_digest_matches_pairs(oracle_mod):
    """orc_join_pp_omp_digest (the whole-window check of joins too large to materialise) ==
    the count and pair_digest of the pairs the same join stores, and == the reference-shaped join."""
    B = (115.5, 117.6, 39.6, 41.1)
    og = oracle_mod.grid(1000, *B)
    ox, oy = oracle_mod.java_random_points(5, 60_000, 116.0, 116.2, 39.8, 39.95)
    qx, qy = oracle_mod.java_random_points(6, 6_000, 116.0, 116.2, 39.8, 39.95)
    st, ref = oracle_mod.join_pp(og, og, ox, oy, qx, qy, 0.001)
    assert st == 0 and len(ref) > 1000
    cnt, dg = oracle_mod.join_pp_digest(og, ox, oy, qx, qy, 0.001, 4)
    assert cnt == len(ref) and dg == oracle_mod.pair_digest(ref)
    assert dg != oracle_mod.pair_digest(ref[1:])  # one pair missing changes it
    swapped = ref.copy()
    swapped[0] = swapped[0][::-1]
    assert dg != oracle_mod.pair_digest(swapped)
