"""GPU: host-resident windows through gf_window_* (the boundary a JNI shim uses).  Uploads run
on the window's own copy stream: they wait for the evaluations already enqueued (which may
still read the old contents) and gf_window_points orders later work after the copy -- so two
device windows double-buffer a stream of host windows.  Columns passed as NULL are not copied
and come back NULL (kNN then refuses the window).  Results equal the oracle's."""
import ctypes as C

import numpy as np
import pytest

from conftest import BEIJING, QPOINT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def pinned_columns(L, arrays):
    n = len(arrays[0])
    p = C.c_void_p()
    assert L.gf_pinned_alloc(8 * n * len(arrays), C.byref(p)) == 0
    v = np.ctypeslib.as_array((C.c_uint8 * (8 * n * len(arrays))).from_address(p.value))
    for j, a in enumerate(arrays):
        v[8 * n * j: 8 * n * (j + 1)] = np.ascontiguousarray(a).view(np.uint8)
    return p, [p.value + 8 * n * j for j in range(len(arrays))]


def test_double_buffered_range_stream(sf, oracle_mod):
    """6 host windows through 2 device windows, upload(i+1) issued before evaluate(i) is even
    enqueued; every window's hits == the oracle's."""
    import torch
    from spatialflink_amd import _lib

    L = _lib.lib()
    ctx = _lib.context(0)
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    n, r, nw = 400_000, 0.05, 6
    hosts = [oracle_mod.java_random_points(500 + i, n, *BEIJING) for i in range(nw)]
    pins = [pinned_columns(L, [x, y]) for x, y in hosts]
    wins = []
    for _ in range(2):
        w = C.c_void_p()
        _lib.check(L.gf_window_create(ctx.handle, n, C.byref(w)), ctx.handle, "window")
        wins.append(w)
    plan = C.c_void_p()
    qx, qy = np.array([QPOINT[0]]), np.array([QPOINT[1]])
    _lib.check(L.gf_range_pp_plan_create(ctx.handle, C.byref(g.c_grid), qx.ctypes.data, qy.ctypes.data, 1, r, 0, 0,
                                         C.byref(plan)), ctx.handle, "plan")
    words = (n + 63) // 64
    bms = [torch.zeros(words, dtype=torch.int64, device="cuda") for _ in range(nw)]
    _lib.check(L.gf_window_upload(wins[0], pins[0][1][0], pins[0][1][1], None, None, n), ctx.handle, "upload")
    for i in range(nw):
        if i + 1 < nw:
            _lib.check(L.gf_window_upload(wins[(i + 1) % 2], pins[i + 1][1][0], pins[i + 1][1][1], None, None, n),
                       ctx.handle, "upload")
        pts = _lib.GfPoints()
        _lib.check(L.gf_window_points(wins[i % 2], C.byref(pts)), ctx.handle, "points")
        assert not pts.objID and not pts.ts  # not uploaded -> NULL
        _lib.check(L.gf_range_run(plan, C.byref(pts), bms[i].data_ptr(), None, None), ctx.handle, "range")
    _lib.check(L.gf_ctx_synchronize(ctx.handle), ctx.handle, "sync")
    for i, (x, y) in enumerate(hosts):
        bits = np.unpackbits(bms[i].cpu().numpy().view(np.uint8), bitorder="little")[:n]
        np.testing.assert_array_equal(np.flatnonzero(bits), oracle_mod.range_pp(og, x, y, qx, qy, r), err_msg=f"{i}")
    L.gf_range_plan_destroy(plan)
    for w in wins:
        L.gf_window_destroy(w)
    for p, _ in pins:
        L.gf_pinned_free(p)


def test_knn_needs_objid_column(sf, oracle_mod):
    from spatialflink_amd import _lib

    L = _lib.lib()
    ctx = _lib.context(0)
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    n, k, r = 300_000, 20, 0.05
    x, y = oracle_mod.java_random_points(77, n, *BEIJING)
    obj = np.arange(n, dtype=np.int64) % 1000
    w = C.c_void_p()
    _lib.check(L.gf_window_create(ctx.handle, n, C.byref(w)), ctx.handle, "window")
    plan = C.c_void_p()
    _lib.check(L.gf_knn_pp_plan_create(ctx.handle, C.byref(g.c_grid), QPOINT[0], QPOINT[1], r, k, 0, C.byref(plan)),
               ctx.handle, "plan")
    oo, od, oi = np.zeros(k, np.int64), np.zeros(k, np.float64), np.zeros(k, np.int64)
    m = C.c_int32()
    pts = _lib.GfPoints()
    # x, y only: the kNN plan refuses the window
    _lib.check(L.gf_window_upload(w, x.ctypes.data, y.ctypes.data, None, None, n), ctx.handle, "upload")
    _lib.check(L.gf_window_points(w, C.byref(pts)), ctx.handle, "points")
    assert L.gf_knn_run(plan, C.byref(pts), oo.ctypes.data, od.ctypes.data, oi.ctypes.data, C.byref(m)) == _lib.GF_ERR_ARG
    # with objID (pageable host memory): the oracle's neighbours
    _lib.check(L.gf_window_upload(w, x.ctypes.data, y.ctypes.data, obj.ctypes.data, None, n), ctx.handle, "upload")
    _lib.check(L.gf_window_points(w, C.byref(pts)), ctx.handle, "points")
    _lib.check(L.gf_knn_run(plan, C.byref(pts), oo.ctypes.data, od.ctypes.data, oi.ctypes.data, C.byref(m)),
               ctx.handle, "knn")
    st, eo, ed, ei = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
    np.testing.assert_array_equal(oo[: m.value], eo)
    np.testing.assert_array_equal(od[: m.value], ed)
    np.testing.assert_array_equal(oi[: m.value], ei)
    L.gf_knn_plan_destroy(plan)
    L.gf_window_destroy(w)


@pytest.mark.parametrize("depth", [1, 3])
def test_knn_mapped_objid_stream(sf, oracle_mod, depth):
    """Host windows at 16 B per point over PCIe (gf_window_upload_mapped): x, y copied, the objID
    column read in place from pinned host memory -- only the candidates' objIDs cross the bus.
    5 host windows double-buffered through 2 device windows (upload(i+1) before evaluate(i)), the
    records written into pinned memory, a plan at depth 1 and at depth 3; every record == the
    oracle's; pageable objID memory is refused (GF_ERR_ARG)."""
    import torch

    from spatialflink_amd import _lib

    L = _lib.lib()
    ctx = _lib.context(0)
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    n, k, r, nw = 1_100_000, 50, 0.5, 5
    hosts = []
    for i in range(nw):
        x, y = oracle_mod.java_random_points(700 + i, n, *BEIJING)
        obj = (np.random.default_rng(i).permutation(n) % (n // 2)).astype(np.int64)
        hosts.append((x, y, obj))
    pins = [pinned_columns(L, list(h)) for h in hosts]
    wins = []
    for _ in range(2):
        w = C.c_void_p()
        _lib.check(L.gf_window_create(ctx.handle, n, C.byref(w)), ctx.handle, "window")
        wins.append(w)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(sf.QueryConfiguration(sf.QueryType.WindowBased), g)
    _, plan = op.plan(0, q, r, k)
    op.set_pipeline(0, q, r, k, depth)
    rec = sf.PinnedRecords(nw, k)
    cols = lambda i: pins[i][1]  # noqa: E731
    try:
        _stream_mapped(sf, oracle_mod, L, ctx, op, q, plan, wins, cols, hosts, rec, og, n, k, r, nw)
    finally:
        ctx.synchronize()
        op.set_pipeline(0, q, r, k, 1)
        for w in wins:
            L.gf_window_destroy(w)
        for p, _ in pins:
            L.gf_pinned_free(p)


def _stream_mapped(sf, oracle_mod, L, ctx, op, q, plan, wins, cols, hosts, rec, og, n, k, r, nw):
    import torch

    from spatialflink_amd import _lib

    _lib.check(L.gf_window_upload_mapped(wins[0], cols(0)[0], cols(0)[1], cols(0)[2], n), ctx.handle, "upload")
    for i in range(nw):
        if i + 1 < nw:
            _lib.check(L.gf_window_upload_mapped(wins[(i + 1) % 2], cols(i + 1)[0], cols(i + 1)[1], cols(i + 1)[2], n),
                       ctx.handle, "upload")
        pts = _lib.GfPoints()
        _lib.check(L.gf_window_points(wins[i % 2], C.byref(pts)), ctx.handle, "points")
        assert pts.objID == cols(i)[2] or pts.objID  # the mapped host column
        _lib.check(L.gf_knn_enqueue(plan, C.byref(pts), C.c_void_p(rec.ptr(i))), ctx.handle, "enqueue")
    op.flush(0, q, r, k)
    torch.cuda.synchronize()
    for i, (x, y, obj) in enumerate(hosts):
        st, o, d, ix = rec.decode(i)
        est, eo, ed, ei = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
        assert st == 0, f"window {i} flagged"
        np.testing.assert_array_equal(o, eo)
        np.testing.assert_array_equal(d, ed)
        np.testing.assert_array_equal(ix, ei)
    x, y, obj = hosts[0]
    assert L.gf_window_upload_mapped(wins[0], x.ctypes.data, y.ctypes.data, obj.ctypes.data, n) == _lib.GF_ERR_ARG
    # the refused call leaves no sticky HIP error behind: the next launch works
    res = op.run(sf.PointWindow.from_numpy(x, y, obj), q, r, k)
    est, eo, ed, ei = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
    np.testing.assert_array_equal(res.objID, eo)
