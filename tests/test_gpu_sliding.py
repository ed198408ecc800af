"""GPU parity of the sliding-window pane engine (gf_knn_sliding_*, gf_pane_bounds) and the
sliding range path: every window that fires is checked against the oracle evaluated on that
window's points from scratch (what the reference's SlidingProcessingTimeWindows operators do),
bit-exact (objID, rank) lists, distances and in-window indices."""
import numpy as np
import pytest

from conftest import BEIJING, QPOINT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def make_stream(oracle_mod, seed, n, t0, t1, gap=None, dup=True):
    x, y = oracle_mod.java_random_points(seed, n, *BEIJING)
    rng = np.random.default_rng(seed)
    ts = np.sort(rng.integers(t0, t1, n)).astype(np.int64)
    if gap is not None:
        keep = ~((ts >= gap[0]) & (ts < gap[1]))
        x, y, ts = x[keep], y[keep], ts[keep]
    m = len(x)
    obj = (rng.permutation(m) % (m // 2 if dup else m)).astype(np.int64)
    return x, y, obj, ts


def batches(sf, x, y, obj, ts, seed, count=7):
    rng = np.random.default_rng(seed + 1)
    cuts = np.sort(rng.choice(np.arange(1, len(x)), count - 1, replace=False))
    b = [0, *cuts.tolist(), len(x)]
    for lo, hi in zip(b[:-1], b[1:]):
        yield sf.PointWindow.from_numpy(x[lo:hi], y[lo:hi], obj[lo:hi], ts[lo:hi])


def expected_windows(ts, size, slide):
    out = []
    s = (int(ts.min()) // slide - size // slide - 1) * slide
    while s <= int(ts.max()):
        if np.any((ts >= s) & (ts < s + size)):
            out.append((s, s + size))
        s += slide
    return out


def conf(sf):
    return sf.QueryConfiguration(sf.QueryType.WindowBased)


@pytest.mark.parametrize("size,slide,k,depth,n,cap,gn", [
    (3000, 1000, 50, 2, 900_000, None, 500),
    (3000, 1000, 50, 1, 900_000, None, 500),
    (4000, 2000, 120, 1, 700_000, None, 500),
    (5000, 3000, 7, 2, 600_000, None, 500),
    (2000, 1000, 50, 2, 400_000, 64, 500),     # every pane overflows: pane-by-pane exact decode
    # C5's shape (BASELINE.json configs[4]): k = 100, 1000 x 1000 grid, size / slide = 2
    (2000, 1000, 100, 2, 1_500_000, None, 1000),
    (2000, 1000, 100, 1, 800_000, None, 1000),
    # any k (KNNQuery.java:216): k in (256, 512] unfused at depth 2, k > 512 on the sorted path with
    # the rank merge of pane records (k = 1000 at C5's grid)
    (3000, 1000, 300, 2, 700_000, None, 500),
    (3000, 1000, 600, 2, 700_000, None, 500),
    (2000, 1000, 1000, 1, 600_000, None, 1000),
])
def test_sliding_knn_matches_oracle(sf, oracle_mod, size, slide, k, depth, n, cap, gn):
    g = sf.UniformGrid(gn, *BEIJING)
    og = oracle_mod.grid(gn, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    x, y, obj, ts = make_stream(oracle_mod, size + slide + k, n, 10_000, 24_000, gap=(15_200, 17_900))
    op = sf.SlidingKNNQuery(conf(sf), g, q, 0.5, k, size_ms=size, slide_ms=slide, pipeline=depth)
    if cap:
        op.op.set_capacity(0, q, 0.5, k, cap)
    got = []
    for b in batches(sf, x, y, obj, ts, size):
        op.push(b)
        got += op.results()
    op.flush()
    got += op.results()
    exp = expected_windows(ts, size, slide)
    assert [(r.windowStart, r.windowEnd) for r in got] == exp
    for r in got:
        m = (ts >= r.windowStart) & (ts < r.windowEnd)
        st, eo, ed, ei = oracle_mod.knn(og, x[m], y[m], obj[m], QPOINT[0], QPOINT[1], 0.5, k)
        assert st == 0
        np.testing.assert_array_equal(r.objID, eo)
        np.testing.assert_array_equal(r.dist, ed)
        np.testing.assert_array_equal(r.idx, ei, err_msg=f"window {r.windowStart}..{r.windowEnd} points {m.sum()} "
                                      f"before {np.count_nonzero(ts < r.windowStart)} panes {sorted(op.panes.items())[:3]}")


def test_pane_bounds_kernel(sf, oracle_mod):
    from spatialflink_amd.windows import pane_bounds

    rng = np.random.default_rng(5)
    ts = np.sort(rng.integers(-50_000, 90_000, 200_003)).astype(np.int64)
    w = sf.PointWindow.from_numpy(np.zeros(len(ts)), np.zeros(len(ts)), None, ts)
    for pane, first, npanes in ((1000, -60, 160), (7, -7200, 900), (100_000, -1, 3)):
        b = pane_bounds(w, pane, first, npanes)
        exp = np.searchsorted(ts, (first + np.arange(npanes + 1)) * pane, side="left")
        np.testing.assert_array_equal(b, exp)


@pytest.mark.parametrize("size,slide,poly", [(3000, 1000, False), (5000, 2000, False), (3000, 1000, True),
                                             (2000, 2000, True)])
def test_sliding_range_matches_oracle(sf, oracle_mod, size, slide, poly):
    """The device pane engine (gf_range_sliding_*): every window holding a point fires with its
    hits = the oracle over that window's points (positions within the window)."""
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    x, y, obj, ts = make_stream(oracle_mod, 77 + size, 500_000, 0, 9_000, gap=(3_000, 4_500))
    if poly:
        rings = oracle_mod.generate_query_polygons(12, BEIJING[0], BEIJING[2], BEIJING[1], BEIJING[3])
        OP = oracle_mod.Polygons(rings)
        polys = [sf.Polygon(r, g) for r in rings]
        op = sf.SlidingRangeQuery(sf.PointPolygonRangeQuery(conf(sf), g), polys, 0.01, size, slide)
        expect = lambda m: oracle_mod.range_ppoly(og, x[m], y[m], OP, 0.01)  # noqa: E731
    else:
        op = sf.SlidingRangeQuery(sf.PointPointRangeQuery(conf(sf), g), [q], 0.05, size, slide)
        expect = lambda m: oracle_mod.range_pp(og, x[m], y[m], [QPOINT[0]], [QPOINT[1]], 0.05)  # noqa: E731
    got = []
    for b in batches(sf, x, y, obj, ts, 3):
        op.push(b)
        got += op.results()
    op.flush()
    got += op.results()
    windows = [(s, e) for s, e, _ in got]
    # every window holding a point fires, the trailing ones included (Flink's final watermark)
    assert windows == expected_windows(ts, size, slide)
    for s, e, hits in got:
        m = (ts >= s) & (ts < e)
        np.testing.assert_array_equal(hits, expect(m))
