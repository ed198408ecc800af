"""Generate the committed golden fixtures (TEST INFRASTRUCTURE).

The reference ships no golden vectors for this path, so the fixtures are
produced here from seeded java.util.Random-compatible inputs by the C oracle
(oracle/geoflink_oracle.c) and, before anything is written, checked against the
independent pure-Python restatement tests/golden/pyref.py.  Re-run with
`python tests/golden/make_golden.py` (it rewrites tests/golden/*.npz).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)

import oracle as O  # noqa: E402
import pyref as P  # noqa: E402

BEIJING = (115.5, 117.6, 39.6, 41.1)
QPOINT = (116.414899, 39.920374)  # README.md:106


def edge_points(g):
    cl = g.cellLength
    ex = [115.5, 117.6, 115.4, 117.7, np.nan, 116.0, 115.5 + 3 * cl, np.inf, -np.inf, 116.0, QPOINT[0], 115.5 - cl]
    ey = [39.6, 41.1, 39.5, 41.2, 40.0, np.nan, 39.6 + 5 * cl, 40.0, 40.0, 39.6 + 71 * cl, QPOINT[1], 39.6 - 2 * cl]
    return np.array(ex), np.array(ey)


def window(seed, n, g):
    x, y = O.java_random_points(seed, n, *BEIJING)
    ex, ey = edge_points(g)
    return np.concatenate([x, ex]), np.concatenate([y, ey])


def main():
    out = {}
    # ---------------- cells ----------------
    for n in (100, 500):
        g = O.grid(n, *BEIJING)
        x, y = window(11, 2000, g)
        cx, cy = O.assign_cells(g, x, y)
        pg = P.Grid(n, *BEIJING)
        assert all(pg.cell(a, b) == (int(c), int(d)) for a, b, c, d in zip(x, y, cx, cy))
        np.savez(os.path.join(HERE, f"cells_n{n}.npz"), x=x, y=y, cx=cx, cy=cy, cellLength=g.cellLength)
        out[f"cells_n{n}"] = len(x)

    g = O.grid(100, *BEIJING)
    pg = P.Grid(100, *BEIJING)
    x, y = window(42, 3000, g)
    objID = (np.arange(len(x)) * 7919 % 100003).astype(np.int64)

    # ---------------- range p-p ----------------
    rec = {"x": x, "y": y}
    qsets = {"q1": [QPOINT], "q3": [QPOINT, (115.55, 40.9), (117.7, 41.0)]}
    for qn, qs in qsets.items():
        qx = np.array([q[0] for q in qs]); qy = np.array([q[1] for q in qs])
        rec[f"{qn}_qx"], rec[f"{qn}_qy"] = qx, qy
        for r in (0.5, 0.05, 0.02, 0.0):
            for ap in (0, 1):
                a = O.range_pp(g, x, y, qx, qy, r, bool(ap))
                b = P.range_pp(pg, x.tolist(), y.tolist(), qs, r, bool(ap))
                assert a.tolist() == b, (qn, r, ap)
                rec[f"{qn}_r{r}_a{ap}"] = a
    np.savez(os.path.join(HERE, "range_pp.npz"), **rec)
    out["range_pp"] = len(rec)

    # ---------------- range p-polygon ----------------
    polys = O.generate_query_polygons(40, 115.5, 39.6, 117.6, 41.1)
    polys.append([[(116.0, 40.0), (116.3, 40.1), (116.1, 40.5), (116.0, 40.0)],
                  [(116.05, 40.05), (116.15, 40.1), (116.1, 40.2), (116.05, 40.05)]])
    polys.append([[(116.5, 40.3), (116.9, 40.3), (116.9, 40.7), (116.7, 40.45), (116.5, 40.7), (116.5, 40.3)]])
    PP = O.Polygons(polys)
    rec = {"x": x, "y": y, "ring_off": PP.ring_off, "vert_off": PP.vert_off, "vx": PP.vx, "vy": PP.vy}
    for r in (0.001, 0.05, 0.3):
        for ap in (0, 1):
            a = O.range_ppoly(g, x, y, PP, r, bool(ap))
            b = P.range_ppoly(pg, x.tolist(), y.tolist(), polys, r, bool(ap))
            assert a.tolist() == b, (r, ap)
            rec[f"r{r}_a{ap}"] = a
    np.savez(os.path.join(HERE, "range_ppoly.npz"), **rec)
    out["range_ppoly"] = len(rec)

    # ---------------- kNN ----------------
    rec = {"x": x, "y": y, "objID": objID}
    dup = objID.copy()
    dup[::3] = dup[::3] % 50  # many repeated objIDs
    rec["objID_dup"] = dup
    for r in (0.5, 0.05, 0.3):
        for k in (1, 50, 100):
            for tag, ob in (("u", objID), ("d", dup)):
                st, oo, od, oi = O.knn(g, x, y, ob, QPOINT[0], QPOINT[1], r, k)
                ref = P.knn_contract(pg, x.tolist(), y.tolist(), ob.tolist(), QPOINT[0], QPOINT[1], r, k)
                assert [(a, b, c) for a, b, c in zip(od.tolist(), oo.tolist(), oi.tolist())] == ref, (r, k, tag)
                rec[f"{tag}_r{r}_k{k}_obj"], rec[f"{tag}_r{r}_k{k}_d"], rec[f"{tag}_r{r}_k{k}_idx"] = oo, od, oi
    np.savez(os.path.join(HERE, "knn.npz"), **rec)
    out["knn"] = len(rec)

    # ---------------- join ----------------
    qx, qy = O.java_random_points(7, 400, *BEIJING)
    rec = {"ox": x, "oy": y, "qx": qx, "qy": qy}
    for r in (0.001, 0.05, 0.0):
        for ap in (0, 1):
            if r == 0.0 and ap:
                continue
            st, pairs = O.join_pp(g, g, x, y, qx, qy, r, bool(ap))
            ref = P.join_pp(pg, pg, x.tolist(), y.tolist(), qx.tolist(), qy.tolist(), r, bool(ap))
            got = sorted(map(tuple, pairs.tolist()))
            assert got == sorted(ref), (r, ap)
            rec[f"r{r}_a{ap}"] = np.array(got, np.int64).reshape(-1, 2)
    np.savez(os.path.join(HERE, "join.npz"), **rec)
    out["join"] = len(rec)
    out["join_ppoly"] = make_join_ppoly()
    print("fixtures written:", out)


def join_ppoly_polygons():
    """The range_ppoly set plus a square straddling the grid's lower-left corner (bbox cells
    outside the grid: keys without validKey when g == 0)."""
    polys = O.generate_query_polygons(40, 115.5, 39.6, 117.6, 41.1)
    polys.append([[(116.0, 40.0), (116.3, 40.1), (116.1, 40.5), (116.0, 40.0)],
                  [(116.05, 40.05), (116.15, 40.1), (116.1, 40.2), (116.05, 40.05)]])
    polys.append([[(116.5, 40.3), (116.9, 40.3), (116.9, 40.7), (116.7, 40.45), (116.5, 40.7), (116.5, 40.3)]])
    polys.append([[(115.45, 39.55), (115.53, 39.55), (115.53, 39.63), (115.45, 39.63), (115.45, 39.55)]])
    return polys


def make_join_ppoly():
    """PointPolygonJoinQuery fixtures: C oracle == pyref before anything is written."""
    g = O.grid(100, *BEIJING)
    pg = P.Grid(100, *BEIJING)
    x, y = window(42, 3000, g)
    polys = join_ppoly_polygons()
    PP = O.Polygons(polys)
    rec = {"x": x, "y": y, "ring_off": PP.ring_off, "vert_off": PP.vert_off, "vx": PP.vx, "vy": PP.vy}
    for r in (0.001, 0.05, 0.3, 0.0):
        for ap in (0, 1):
            a = O.join_ppoly(g, g, x, y, PP, r, bool(ap))
            got = sorted(map(tuple, a.tolist()))
            ref = P.join_ppoly(pg, pg, x.tolist(), y.tolist(), polys, r, bool(ap))
            assert got == ref, (r, ap, len(got), len(ref))
            rec[f"r{r}_a{ap}"] = np.array(got, np.int64).reshape(-1, 2)
    np.savez(os.path.join(HERE, "join_ppoly.npz"), **rec)
    return len(rec)


if __name__ == "__main__":
    if sys.argv[1:] == ["join_ppoly"]:
        print("fixtures written:", {"join_ppoly": make_join_ppoly()})
    else:
        main()
