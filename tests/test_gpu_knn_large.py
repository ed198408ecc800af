"""GPU: kNN with k > 512 (the reference's PriorityQueue takes any k, KNNQuery.java:216).  Such
plans keep every candidate within r and derive the record from two stable device radix sorts
((objID, d, idx) -> first of each objID -> (d, objID, idx)); the exact re-evaluation of a
flagged window takes the same path.  Results == the oracle's contract (orc_knn_contract /
orc_knn_ppoly_contract), bit-exact, for point and polygon queries, duplicate objIDs, fewer
distinct objIDs than k, clustered input.  The sorted path reads its counts on the device, so
windows queue back to back (depths 2 / 3 accept k > 512); k in (256, 512] pipelines unfused (the
standalone select, lanes alternating over two streams at depth 3); records of any k merge on the
device (gf_knn_merge_dev(_batch): ranks by binary search + objID dedupe for k > 512)."""
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


def check(res, oo, od, oi):
    np.testing.assert_array_equal(res.objID, oo)
    np.testing.assert_array_equal(res.dist.view(np.int64), od.view(np.int64))
    np.testing.assert_array_equal(res.idx, oi)


@pytest.mark.parametrize("n,grid_n,r,k,dup", [
    (2_000_001, 500, 0.05, 513, False),
    (2_000_001, 500, 0.5, 5_000, True),
    (1_000_000, 100, 0.3, 100_000, True),    # more than the distinct objIDs within r? checked below
    (300_000, 1000, 0.004, 2_000, False),    # fewer candidates than k
    (0, 500, 0.5, 1000, False),
])
def test_knn_large_k(sf, oracle_mod, n, grid_n, r, k, dup):
    g = sf.UniformGrid(grid_n, *BEIJING)
    og = oracle_mod.grid(grid_n, *BEIJING)
    x, y = oracle_mod.java_random_points(grid_n + k, n, *BEIJING)
    obj = np.random.default_rng(k).permutation(n).astype(np.int64)
    if dup:
        obj %= max(1, n // 7)
    q = sf.Point("q", *QPOINT, 0, g)
    res = sf.PointPointKNNQuery(conf(sf), g).run(sf.PointWindow.from_numpy(x, y, obj), q, r, k)
    st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
    check(res, oo, od, oi)
    if n == 300_000:
        assert len(oo) < k


def test_knn_large_k_clustered_and_continuous(sf, oracle_mod):
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)  # one plan, several windows (buffers reused / grown)
    for seed, n in ((3, 500_000), (4, 1_500_000), (5, 800_000)):
        x, y = sf.synthetic_clustered(seed, n, *BEIJING, centers=[QPOINT])
        obj = np.arange(n, dtype=np.int64) % (n // 2)
        res = op.run(sf.PointWindow.from_numpy(x, y, obj), q, 0.1, 3_000)
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.1, 3_000)
        check(res, oo, od, oi)


def test_polygon_knn_large_k(sf, oracle_mod):
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    h = 0.01
    ring = [(QPOINT[0] - h, QPOINT[1] - h), (QPOINT[0] + h, QPOINT[1] - h), (QPOINT[0] + h, QPOINT[1] + h),
            (QPOINT[0] - h, QPOINT[1] + h), (QPOINT[0] - h, QPOINT[1] - h)]
    P = sf.Polygon([ring], g)
    x, y = oracle_mod.java_random_points(17, 1_200_000, *BEIJING)
    obj = (np.arange(len(x)) % 400_000).astype(np.int64)
    res = sf.PointPolygonKNNQuery(conf(sf), g).run(sf.PointWindow.from_numpy(x, y, obj), P, 0.2, 1_500)
    m, eo, ed, ei = oracle_mod.knn_ppoly(og, x, y, obj, oracle_mod.Polygons([P.rings]), 0.2, 1_500)
    check(res, eo, ed, ei)


@pytest.mark.parametrize("k,depth", [(700, 1), (700, 2), (700, 3), (700, 4), (300, 2), (300, 3), (512, 3), (400, 4)])
def test_knn_large_k_queued_windows(sf, oracle_mod, k, depth):
    """Several windows enqueued back to back with no host read in between (records written by the
    kernels straight into pinned host memory), then one flush: each record == the oracle's.
    Window sizes shrink and grow (candidate buffers regrown in stream order).  k > 512: the sorted
    path; k in (256, 512]: the unfused pipeline (depth 3: two lanes on two streams)."""
    import torch

    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    r = 0.2
    data = []
    for seed, n in ((31, 900_000), (32, 200_000), (33, 1_300_000), (34, 0), (35, 600_000), (36, 1_100_000)):
        x, y = oracle_mod.java_random_points(seed, n, *BEIJING)
        obj = (np.arange(n) % max(1, n // 3)).astype(np.int64)
        data.append((x, y, obj, sf.PointWindow.from_numpy(x, y, obj)))
    op.set_pipeline(0, q, r, k, depth)
    order = [0, 1, 2, 3, 4, 2, 0, 5, 5, 2]
    rec = sf.PinnedRecords(len(order), k)
    for i, j in enumerate(order):
        op.enqueue(data[j][3], q, r, k, rec.ptr(i))
    op.flush(0, q, r, k)
    torch.cuda.synchronize()
    for i, j in enumerate(order):
        x, y, obj, w = data[j]
        res = op.finish(w, q, r, k, rec.raw(i))
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
        check(res, oo, od, oi)
    op.set_pipeline(0, q, r, k, 1)


@pytest.mark.parametrize("k,layout", [(600, 0), (600, 1), (2_000, 0)])
def test_knn_merge_any_k(sf, oracle_mod, k, layout):
    """Sharded windows at k > 512: each shard's record (the sorted path, index bases so idx is
    global), merged by ONE gf_knn_merge_dev_batch launch (both layouts) == each window evaluated
    whole.  objIDs repeat within and across shards, and exact distance ties across shards (points
    duplicated into two shards with different objIDs / the same objID) must merge by (d, objID, idx)."""
    import torch

    from spatialflink_amd import _lib

    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    S, W = 4, 3
    rb = sf.spatialOperators.knn_record_bytes(k)
    recs = torch.zeros(S * W * rb, dtype=torch.uint8, device="cuda")
    expect = []
    ops = [sf.PointPointKNNQuery(conf(sf), g) for _ in range(S)]
    for wi in range(W):
        x, y = oracle_mod.java_random_points(500 + wi, 400_000, *BEIJING)
        obj = (np.random.default_rng(wi).permutation(len(x)) % 150_000).astype(np.int64)
        # exact ties: a block of points copied to the other half of the window (other shards)
        x[200_000:201_000], y[200_000:201_000] = x[:1000], y[:1000]
        obj[200_500:201_000] = obj[500:1000]
        expect.append(oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.3, k))
        for s, ix in enumerate(np.array_split(np.arange(len(x)), S)):
            ctx, plan = ops[s].plan(0, q, 0.3, k)
            _lib.check(_lib.lib().gf_knn_plan_set_index_base(plan, int(ix[0])), ctx.handle, "base")
            slot = s * W + wi if layout == 0 else wi * S + s
            ops[s].enqueue(sf.PointWindow.from_numpy(x[ix], y[ix], obj[ix]), q, 0.3, k, recs[slot * rb:(slot + 1) * rb])
    out = torch.zeros(W * rb, dtype=torch.uint8, device="cuda")
    ctx = _lib.context(0)
    _lib.check(_lib.lib().gf_knn_merge_dev_batch(ctx.handle, k, recs.data_ptr(), S, W, layout, out.data_ptr()),
               ctx.handle, "merge batch")
    raw = out.cpu().numpy().tobytes()
    for wi in range(W):
        st, o, d, i = sf.spatialOperators.decode_knn_record(raw[wi * rb:(wi + 1) * rb], k)
        est, eo, ed, ei = expect[wi]
        assert st == 0 and len(eo) == min(k, len(eo))
        np.testing.assert_array_equal(o, eo)
        np.testing.assert_array_equal(d.view(np.int64), ed.view(np.int64))
        np.testing.assert_array_equal(i, ei)
    # one window through gf_knn_merge_dev (shard-major records of window 0 are contiguous at layout 0)
    if layout == 0:
        one = torch.zeros(rb, dtype=torch.uint8, device="cuda")
        win0 = torch.cat([recs[(s * W) * rb:(s * W + 1) * rb] for s in range(S)])
        _lib.check(_lib.lib().gf_knn_merge_dev(ctx.handle, k, win0.data_ptr(), S, one.data_ptr()), ctx.handle, "merge")
        st, o, d, i = sf.spatialOperators.decode_knn_record(one.cpu().numpy().tobytes(), k)
        np.testing.assert_array_equal(o, expect[0][1])
        np.testing.assert_array_equal(i, expect[0][3])
