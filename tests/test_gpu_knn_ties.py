"""GPU: kNN windows whose k-th distance bin alone overflows the select's sort area -- a dense
ring of nearly equal distances, points stacked on one spot (equal non-zero distances), points
inside a query polygon (d = 0).  The select splits that bin by a second histogram (distance
bits, or the objID key when every distance in it is equal) instead of streaming every
candidate against a running list (KNNQuery.java:216-251 orders by (distance, objID) after the
objID dedupe).  Records == the oracle's contract bit-exact at depths 1, 2 and 3."""
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


def tie_window(oracle_mod, kind, seed, n_bg=1_000_000, n_tie=3000):
    rng = np.random.default_rng(seed)
    x, y = oracle_mod.java_random_points(seed, n_bg, *BEIJING)
    if kind == "ring":  # distances in [0.01, 0.01 + 1e-6]: one log bin, all different
        a = rng.uniform(0, 2 * np.pi, n_tie)
        rr = 0.01 + rng.uniform(0, 1e-6, n_tie)
        tx, ty = QPOINT[0] + rr * np.cos(a), QPOINT[1] + rr * np.sin(a)
    elif kind == "stack":  # one spot: every distance equal and non-zero
        tx, ty = np.full(n_tie, QPOINT[0] + 0.003), np.full(n_tie, QPOINT[1] - 0.002)
    else:  # inside the query point's cell neighbourhood at distance 0 (the query point itself)
        tx, ty = np.full(n_tie, QPOINT[0]), np.full(n_tie, QPOINT[1])
    x, y = np.concatenate([x, tx]), np.concatenate([y, ty])
    p = rng.permutation(len(x))  # ties scattered over the window
    x, y = x[p], y[p]
    obj = (rng.permutation(len(x)) % (len(x) * 2 // 3)).astype(np.int64)  # some duplicate objIDs
    return x, y, obj


def check(res, oo, od, oi):
    np.testing.assert_array_equal(res.objID, oo)
    np.testing.assert_array_equal(res.dist.view(np.int64), od.view(np.int64))
    np.testing.assert_array_equal(res.idx, oi)


@pytest.mark.parametrize("kind", ["ring", "stack", "zero"])
@pytest.mark.parametrize("k", [50, 300])
def test_knn_tie_bin(sf, oracle_mod, kind, k):
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    for seed in (1, 2):  # the second window runs with the first one's hint
        x, y, obj = tie_window(oracle_mod, kind, seed)
        res = op.run(sf.PointWindow.from_numpy(x, y, obj), q, 0.5, k)
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
        check(res, oo, od, oi)


@pytest.mark.parametrize("depth", [2, 3])
def test_knn_tie_bin_pipelined(sf, oracle_mod, depth):
    """The fused select (block 0 of the next window's scan, 256-entry sort area)."""
    import torch

    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    k = 40
    data = []
    for seed, kind in ((3, "ring"), (4, "stack"), (5, "zero"), (6, "ring")):
        x, y, obj = tie_window(oracle_mod, kind, seed, n_tie=1500)
        data.append((x, y, obj, sf.PointWindow.from_numpy(x, y, obj)))
    op.set_pipeline(0, q, 0.5, k, depth)
    order = [0, 1, 2, 3, 1, 0, 2]
    rec = sf.PinnedRecords(len(order), k)
    for i, j in enumerate(order):
        op.enqueue(data[j][3], q, 0.5, k, rec.ptr(i))
    op.flush(0, q, 0.5, k)
    torch.cuda.synchronize()
    for i, j in enumerate(order):
        x, y, obj, w = data[j]
        res = op.finish(w, q, 0.5, k, rec.raw(i))
        st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
        check(res, oo, od, oi)
    op.set_pipeline(0, q, 0.5, k, 1)


def test_knn_capacity_grown_after_depth4(sf, oracle_mod):
    """gf_knn_plan_set_capacity after gf_knn_plan_set_pipeline(4) regrows EVERY lane (depth 4 runs
    six lanes on three streams): the plan starts at a 1024-candidate capacity, goes to depth 4,
    then to 16384; 18 windows of ~3000 stacked ties each (more than the old capacity) cycle over
    all six lanes.  Every record == the oracle (flagged ones re-evaluated by finish()), and once
    each lane has adapted its hint (the last six windows: the third visit of every lane) every
    record is final -- a lane left at the old capacity would overflow (status 1) there."""
    import torch

    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(conf(sf), g)
    k = 40
    op.set_capacity(0, q, 0.5, k, 1024)
    op.set_pipeline(0, q, 0.5, k, 4)
    op.set_capacity(0, q, 0.5, k, 16384)
    data = []
    for seed, kind in ((7, "stack"), (8, "zero"), (9, "stack")):
        x, y, obj = tie_window(oracle_mod, kind, seed, n_bg=400_000, n_tie=3000)
        data.append((x, y, obj, sf.PointWindow.from_numpy(x, y, obj)))
    order = [0, 1, 2] * 6
    rec = sf.PinnedRecords(len(order), k)
    try:
        for i, j in enumerate(order):
            op.enqueue(data[j][3], q, 0.5, k, rec.ptr(i))
        op.flush(0, q, 0.5, k)
        torch.cuda.synchronize()
        for i, j in enumerate(order):
            raw = rec.raw(i)
            status, n = np.frombuffer(raw[:8], np.int32)
            if i >= len(order) - 6:
                assert status == 0, f"window {i} flagged (status {status}): a lane kept the old capacity"
            x, y, obj, w = data[j]
            res = op.finish(w, q, 0.5, k, raw)
            st, oo, od, oi = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
            check(res, oo, od, oi)
    finally:
        op.set_pipeline(0, q, 0.5, k, 1)
