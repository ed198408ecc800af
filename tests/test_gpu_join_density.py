"""GPU: the point-point join at C4's OCCUPANCY (BASELINE.json configs[3]: 10M ordinary x 1M query
points on the 1000 x 1000 Beijing grid, r = 0.001 -> ~14 ordinary and ~1.4 query points per cell,
~10 pairs per query point), whole windows compared pair for pair with the oracle
(join/PointPointJoinQuery.java:148-182, JoinQuery.java:73-90).

The C4 bench window spreads 10M points over the whole grid; here 400K x 40K points are confined to
a 0.42 x 0.30 degree box (200 x 143 cells), which is the same density per cell, so the band probe's
staged-band sizes, per-block regions, spill and the fix-up copy run at
the bench's occupancy.  Consecutive windows of DIFFERENT densities run on one context: each call
sizes its output regions from the previous call's pairs per point of every block, so a denser
window after a sparse one overflows its regions (the overflow area in the spill), a sparser one
leaves long region tails (holes filled by the fix-up copy)."""
import ctypes as C

import numpy as np
import pytest

from conftest import BEIJING

pytestmark = pytest.mark.gpu

BOX = (116.0, 116.42, 39.8, 40.1)  # 200 x 143 cells of the 1000-grid (cell side 0.0021)
R = 0.001


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def win(sf, x, y):
    return sf.PointWindow.from_numpy(np.ascontiguousarray(x), np.ascontiguousarray(y))


def sorted_pairs(p):
    p = np.asarray(p, np.int64).reshape(-1, 2)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


def window(oracle_mod, sf, kind, seed):
    """(ordinary x, y, query x, y) of one window: `kind` = density factor, or "clustered"."""
    if kind == "clustered":
        ox, oy = sf.synthetic_clustered(seed, 400_000, *BOX, n_centers=6, sigma=0.004, frac=0.6)
        qx, qy = sf.synthetic_clustered(seed, 40_000, *BOX, n_centers=6, sigma=0.004, frac=0.6)
        return ox, oy, qx, qy
    n = int(400_000 * kind)
    ox, oy = oracle_mod.java_random_points(seed, n, BOX[0], BOX[1], BOX[2], BOX[3])
    qx, qy = oracle_mod.java_random_points(seed + 1, n // 10, BOX[0], BOX[1], BOX[2], BOX[3])
    return ox, oy, qx, qy


def expected(oracle_mod, og, ox, oy, qx, qy):
    return oracle_mod.join_pp_mt(og, og, ox, oy, qx, qy, R, 8, optimized=True)


def test_join_c4_density_reference_shaped(sf, oracle_mod):
    """One window at C4 occupancy against the reference-shaped oracle (string cell keys,
    replicated query side, per-cell nested loop) -- it also pins the optimised OpenMP oracle the
    other windows use."""
    g = sf.UniformGrid(1000, *BEIJING)
    og = oracle_mod.grid(1000, *BEIJING)
    ox, oy, qx, qy = window(oracle_mod, sf, 1.0, 401)
    st, ref = oracle_mod.join_pp(og, og, ox, oy, qx, qy, R)
    assert st == 0
    ref = sorted_pairs(ref)
    occ = len(ox) / (200 * 143)
    assert 13 < occ < 15 and len(ref) > 300_000  # ~14 ordinary points per cell, ~10 pairs per query point
    np.testing.assert_array_equal(expected(oracle_mod, og, ox, oy, qx, qy), ref)
    got = sf.PointPointJoinQuery(sf.QueryConfiguration(sf.QueryType.WindowBased), g, g).run(win(sf, ox, oy),
                                                                                           win(sf, qx, qy), R)
    np.testing.assert_array_equal(got, ref)


def test_join_c4_density_window_sequence(sf, oracle_mod):
    """Windows of density 1, 2, 0.25, clustered, 1 on ONE context through the raw C ABI with the
    capacity set to exactly the window's pair count: regions sized from the previous window's
    per-block history overflow (denser) or leave holes (sparser), and every window must still
    complete in ONE call (GF_OK, every pair): GF_ERR_CAPACITY only when the pairs exceed cap."""
    import torch

    from spatialflink_amd import _lib

    L = _lib.lib()
    g = sf.UniformGrid(1000, *BEIJING)
    og = oracle_mod.grid(1000, *BEIJING)
    ctx = _lib.context(0)
    retries = 0
    for j, kind in enumerate((1.0, 2.0, 0.25, "clustered", 1.0, 2.0)):
        ox, oy, qx, qy = window(oracle_mod, sf, kind, 410 + 3 * j)
        exp = expected(oracle_mod, og, ox, oy, qx, qy)
        assert len(exp) > 0
        wo, wq = win(sf, ox, oy), win(sf, qx, qy)
        po, pq = wo.c_struct(), wq.c_struct()
        cap = len(exp)
        for attempt in range(3):
            buf = torch.full((2 * cap + 2,), -1, dtype=torch.int32, device="cuda")
            n = C.c_int64()
            st = L.gf_join_pp(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), R, 0, 0,
                              buf.data_ptr(), cap, C.byref(n))
            if st == _lib.GF_ERR_CAPACITY:  # (a failure: counted and reported below)
                retries += 1
                continue
            _lib.check(st, ctx.handle, "gf_join_pp")
            break
        assert st == 0 and n.value == len(exp), f"window {j} ({kind}): {n.value} pairs, expected {len(exp)}"
        got = buf[: 2 * len(exp)].cpu().numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
        np.testing.assert_array_equal(sorted_pairs(got), exp, err_msg=f"window {j} ({kind})")
        assert buf[-2:].cpu().tolist() == [-1, -1]  # nothing written past cap
    # cap == the exact count: no window may be answered GF_ERR_CAPACITY
    assert retries == 0, f"{retries} GF_ERR_CAPACITY answers for windows whose pairs fit"
    # a buffer one pair short: GF_ERR_CAPACITY with the exact count
    ox, oy, qx, qy = window(oracle_mod, sf, 1.0, 499)
    exp = expected(oracle_mod, og, ox, oy, qx, qy)
    wo, wq = win(sf, ox, oy), win(sf, qx, qy)
    po, pq = wo.c_struct(), wq.c_struct()
    buf = torch.full((2 * len(exp),), -1, dtype=torch.int32, device="cuda")
    n = C.c_int64()
    st = L.gf_join_pp(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), R, 0, 0,
                      buf.data_ptr(), len(exp) - 1, C.byref(n))
    assert st == _lib.GF_ERR_CAPACITY and n.value == len(exp)
    assert buf[-2:].cpu().tolist() == [-1, -1]  # nothing written past cap


def test_join_c4_density_async_queue(sf, oracle_mod):
    """The same densities queued back to back with gf_join_pp_async on one context (no host wait
    between windows, counts in device memory), each with capacity = its exact pair count; a
    window completes in its one call (no re-run) and == the oracle."""
    import torch

    from spatialflink_amd import _lib

    L = _lib.lib()
    g = sf.UniformGrid(1000, *BEIJING)
    og = oracle_mod.grid(1000, *BEIJING)
    ctx = _lib.context(0)
    kinds = (0.25, 2.0, 1.0, "clustered", 0.5)
    data = []
    for j, kind in enumerate(kinds):
        ox, oy, qx, qy = window(oracle_mod, sf, kind, 440 + 3 * j)
        exp = expected(oracle_mod, og, ox, oy, qx, qy)
        data.append((win(sf, ox, oy), win(sf, qx, qy), exp))
    bufs = [torch.full((2 * len(e) + 2,), -1, dtype=torch.int32, device="cuda") for _, _, e in data]
    totals = torch.zeros(len(data), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    structs = [(wo.c_struct(), wq.c_struct()) for wo, wq, _ in data]
    for j, ((po, pq), (_, _, e)) in enumerate(zip(structs, data)):
        _lib.check(L.gf_join_pp_async(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), R, 0,
                                      0, bufs[j].data_ptr(), len(e), totals[j].data_ptr()), ctx.handle, "async")
    ctx.synchronize()
    for j, (wo, wq, e) in enumerate(data):
        n = int(totals[j].item())  # one call per window: capacity == the pairs always completes
        assert n == len(e), f"window {j} ({kinds[j]}): {n} pairs, expected {len(e)}"
        got = bufs[j][: 2 * n].cpu().numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
        np.testing.assert_array_equal(sorted_pairs(got), e, err_msg=f"window {j} ({kinds[j]})")
        assert bufs[j][-2:].cpu().tolist() == [-1, -1]


def test_join_count_only_call(sf, oracle_mod):
    """A counting call (pairs NULL, cap 0) returns the exact pair count as GF_ERR_CAPACITY, and 0
    with GF_OK for a window without pairs (the region extent must not count as lost
    pairs)."""
    from spatialflink_amd import _lib

    L = _lib.lib()
    g = sf.UniformGrid(1000, *BEIJING)
    og = oracle_mod.grid(1000, *BEIJING)
    ctx = _lib.context(0)
    ox, oy, qx, qy = window(oracle_mod, sf, 1.0, 470)
    exp = expected(oracle_mod, og, ox, oy, qx, qy)
    wo, wq = win(sf, ox, oy), win(sf, qx, qy)
    po, pq = wo.c_struct(), wq.c_struct()
    n = C.c_int64()
    st = L.gf_join_pp(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), R, 0, 0, None, 0,
                      C.byref(n))
    assert st == _lib.GF_ERR_CAPACITY and n.value == len(exp)
    # no pairs: the query side far away from every ordinary point
    far = win(sf, qx + 0.6, qy)
    pf = far.c_struct()
    st = L.gf_join_pp(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pf), R, 0, 0, None, 0,
                      C.byref(n))
    assert st == 0 and n.value == 0
