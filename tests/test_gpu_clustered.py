"""GPU: the clustered variant of the synthetic source (Gaussian hot spots,
sigma = 0.01 deg) through every query kind, against the oracle.  Skew is what stresses the
kNN threshold sample (hundreds of thousands of points within a few cells of the query), the
range scan's candidate queue (a hot cell on the query's candidate ring), the join's dense rows
(query rows past the LDS budget take the global-memory probe) and the point-polygon tests.
The first hot spot sits on the query point (PointPointKNNQuery / range anchors as in
test_gpu_parity)."""
import numpy as np
import pytest

from conftest import BEIJING, QPOINT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def conf(sf):
    return sf.QueryConfiguration(sf.QueryType.WindowBased)


def win(sf, x, y, obj=None):
    return sf.PointWindow.from_numpy(np.ascontiguousarray(x), np.ascontiguousarray(y), obj)


def pts(sf, seed, n, **kw):
    return sf.synthetic_clustered(seed, n, *BEIJING, centers=[QPOINT], **kw)


def sorted_pairs(p):
    p = np.asarray(p, np.int64).reshape(-1, 2)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


@pytest.mark.parametrize("grid_n,r,k", [(500, 0.5, 50), (500, 0.05, 50), (1000, 0.01, 100), (100, 0.3, 7)])
def test_knn_clustered_sampled(sf, oracle_mod, grid_n, r, k):
    """2M points, 80% in 8 hot spots, one on the query point: the k nearest are all inside the
    query's cell, the candidate ring is dense."""
    g = sf.UniformGrid(grid_n, *BEIJING)
    og = oracle_mod.grid(grid_n, *BEIJING)
    N = 2_000_001
    x, y = pts(sf, grid_n + k, N)
    obj = np.random.default_rng(k).permutation(N).astype(np.int64) % (N // 3)  # repeated objIDs
    q = sf.Point("q", *QPOINT, 0, g)
    res = sf.PointPointKNNQuery(conf(sf), g).run(win(sf, x, y, obj), q, r, k)
    st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
    np.testing.assert_array_equal(res.objID, oo)
    np.testing.assert_array_equal(res.dist, od)
    np.testing.assert_array_equal(res.idx, oi)


@pytest.mark.parametrize("r", [0.5, 0.05, 0.005])
def test_range_pp_clustered(sf, oracle_mod, r):
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    x, y = pts(sf, 7, 1_000_000)
    q = sf.Point("q", *QPOINT, 0, g)
    res = sf.PointPointRangeQuery(conf(sf), g).run(win(sf, x, y), [q], r)
    np.testing.assert_array_equal(np.sort(res.indices().astype(np.int64)),
                                  oracle_mod.range_pp(og, x, y, [QPOINT[0]], [QPOINT[1]], r))


def test_range_ppoly_clustered(sf, oracle_mod):
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    raw = oracle_mod.generate_query_polygons(1000, BEIJING[0], BEIJING[2], BEIJING[1], BEIJING[3])
    polys = [sf.Polygon(rings, g) for rings in raw]
    # hot spots on the polygon block (the generated squares sit at the grid's lower-left corner)
    x, y = sf.synthetic_clustered(8, 1_500_000, *BEIJING, centers=[(115.55, 39.65), (115.6, 39.7)], n_centers=4)
    res = sf.PointPolygonRangeQuery(conf(sf), g).run(win(sf, x, y), polys, 0.001)
    np.testing.assert_array_equal(np.sort(res.indices().astype(np.int64)),
                                  oracle_mod.range_ppoly(og, x, y, oracle_mod.Polygons(raw), 0.001))


@pytest.mark.parametrize("grid_n,r", [(1000, 0.001), (500, 0.004)])
def test_join_clustered(sf, oracle_mod, grid_n, r):
    """Both sides clustered on the same hot spots: dense query rows exceed the probe's LDS budget
    (global-memory tasks) next to ordinary rows that fit."""
    g = sf.UniformGrid(grid_n, *BEIJING)
    og = oracle_mod.grid(grid_n, *BEIJING)
    ox, oy = pts(sf, 61, 300_000)
    qx, qy = pts(sf, 61, 60_000, frac=0.9)  # same seed: same centres
    got = sf.PointPointJoinQuery(conf(sf), g, g).run(win(sf, ox, oy), win(sf, qx, qy), r)
    st, pairs = oracle_mod.join_pp(og, og, ox, oy, qx, qy, r)
    assert st == 0 and len(pairs) > 100_000
    np.testing.assert_array_equal(sorted_pairs(got), sorted_pairs(pairs))
