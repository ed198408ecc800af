"""Independent pure-Python restatement of the reference hot path (TEST INFRASTRUCTURE).

Written separately from the C oracle (oracle/geoflink_oracle.c) so the two can be
diffed when the golden fixtures are generated (tests/golden/make_golden.py).  Small
inputs only (pure-Python loops).  Follows the same reference files:
  UniformGrid.java:74-85,165-229,368-445; HelperClass.java:54-63,104-143,263-276;
  PointPointRangeQuery.java:111-187; PointPolygonRangeQuery.java:134-205;
  PointPointKNNQuery.java:132-201 + KNNQuery.java:213-272 (build contract, A7);
  JoinQuery.java:73-90 + PointPointJoinQuery.java:124-183;
  JoinQuery.java:93-115 + PointPolygonJoinQuery.java:154-213;
  JTS 1.16.1 DistanceOp / Distance.pointToSegment / RayCrossingCounter (restated).
Exact orientation signs use fractions.Fraction (not the oracle's expansion arithmetic).
Metric: sqrt(dx*dx + dy*dy) only.
"""
from __future__ import annotations

import math
from fractions import Fraction


def jint(v: float) -> int:
    if v != v:
        return 0
    if v >= 2147483647.0:
        return 2147483647
    if v <= -2147483648.0:
        return -2147483648
    return int(v)


def _jfloor(v):
    """(int) Math.floor(v) in Java, including NaN and infinities"""
    return jint(v) if (v != v or math.isinf(v)) else jint(math.floor(v))


class Grid:
    def __init__(self, n, minX, maxX, minY, maxY):
        self.n = n
        self.minX, self.maxX, self.minY, self.maxY = minX, maxX, minY, maxY
        self.cl = (maxX - minX) / n

    def cell(self, x, y):
        return _jfloor((x - self.minX) / self.cl), _jfloor((y - self.minY) / self.cl)

    def valid(self, i, j):
        return 0 <= i < self.n and 0 <= j < self.n

    def g_layers(self, r):
        return _jfloor(r / (self.cl * math.sqrt(2)) - 1)

    def c_layers(self, r):
        v = r / self.cl
        return jint(v) if (v != v or math.isinf(v)) else jint(math.ceil(v))


def cell_id(i, j):
    return "%05d%05d" % (i, j) if i >= 0 and j >= 0 else _java_fmt(i) + _java_fmt(j)


def _java_fmt(v):
    return ("-" + ("%04d" % -v)) if v < 0 else "%05d" % v


def parse_id(s):
    def pint(t):
        k = 0
        while k + 1 < len(t) and t[k] == "0":
            k += 1
        return int(t[k:])
    return pint(s[:5]), pint(s[5:])


def g_set(grid, r, cid):
    g = grid.g_layers(r)
    out = set()
    if g == 0:
        out.add(cid)
    elif g > 0:
        qx, qy = parse_id(cid)
        for i in range(max(qx - g, 0), min(qx + g, grid.n - 1) + 1):
            for j in range(max(qy - g, 0), min(qy + g, grid.n - 1) + 1):
                out.add(cell_id(i, j))
    return out


def c_set(grid, r, cid, G):
    c = grid.c_layers(r)
    out = set()
    if c > 0:
        qx, qy = parse_id(cid)
        for i in range(max(qx - c, 0), min(qx + c, grid.n - 1) + 1):
            for j in range(max(qy - c, 0), min(qy + c, grid.n - 1) + 1):
                k = cell_id(i, j)
                if k not in G:
                    out.add(k)
    return out


def dist(x1, y1, x2, y2):
    dx = x1 - x2
    dy = y1 - y2
    return math.sqrt(dx * dx + dy * dy)


def range_pp(grid, xs, ys, qs, r, approximate=False):
    G, C = set(), set()
    for (qx, qy) in qs:
        cid = cell_id(*grid.cell(qx, qy))
        G |= g_set(grid, r, cid)
        C |= c_set(grid, r, cid, G)
    out = []
    for i, (x, y) in enumerate(zip(xs, ys)):
        k = cell_id(*grid.cell(x, y))
        if k in G:
            out.append(i)
        elif k in C:
            for (qx, qy) in qs:
                if approximate:
                    out.append(i)
                elif dist(qx, qy, x, y) <= r:
                    out.append(i)
                    break
    return out


def _seg(px, py, ax, ay, bx, by):
    if ax == bx and ay == by:
        return dist(px, py, ax, ay)
    len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay)
    rr = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2
    if rr <= 0.0:
        return dist(px, py, ax, ay)
    if rr >= 1.0:
        return dist(px, py, bx, by)
    s = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2
    return abs(s) * math.sqrt(len2)


def _sgn_det(x1, y1, x2, y2):
    v = Fraction(x1) * Fraction(y2) - Fraction(y1) * Fraction(x2)
    return (v > 0) - (v < 0)


def _ring_loc(px, py, ring):
    xs = [v[0] for v in ring]
    ys = [v[1] for v in ring]
    if px > max(xs) or px < min(xs) or py > max(ys) or py < min(ys):
        return "E"
    cross = 0
    for i in range(1, len(ring)):
        (p1x, p1y), (p2x, p2y) = ring[i], ring[i - 1]
        if p1x < px and p2x < px:
            continue
        if px == p2x and py == p2y:
            return "B"
        if p1y == py and p2y == py:
            if min(p1x, p2x) <= px <= max(p1x, p2x):
                return "B"
            continue
        if (p1y > py and p2y <= py) or (p2y > py and p1y <= py):
            s = _sgn_det(p1x - px, p1y - py, p2x - px, p2y - py)
            if s == 0:
                return "B"
            if (p2y - py) < (p1y - py):
                s = -s
            if s > 0:
                cross += 1
    return "I" if cross % 2 else "E"


def _env_dist(ring, px, py):
    minx, maxx = min(v[0] for v in ring), max(v[0] for v in ring)
    miny, maxy = min(v[1] for v in ring), max(v[1] for v in ring)
    if not (px > maxx or px < minx or py > maxy or py < miny):
        return 0.0
    dx = px - maxx if maxx < px else (minx - px if minx > px else 0.0)
    dy = py - maxy if maxy < py else (miny - py if miny > py else 0.0)
    if dx == 0.0:
        return dy
    if dy == 0.0:
        return dx
    return math.sqrt(dx * dx + dy * dy)


def point_polygon_distance(px, py, rings):
    loc = _ring_loc(px, py, rings[0]) if px == px else "E"  # NaN x: containment skipped
    if loc == "B":
        return 0.0
    if loc == "I":
        inside = True
        for h in rings[1:]:
            hl = _ring_loc(px, py, h)
            if hl == "I":
                inside = False
                break
            if hl == "B":
                return 0.0
        if inside:
            return 0.0
    md = 1.7976931348623157e308
    for ring in rings:
        if _env_dist(ring, px, py) > md:
            continue
        for i in range(len(ring) - 1):
            d = _seg(px, py, ring[i][0], ring[i][1], ring[i + 1][0], ring[i + 1][1])
            if d < md:
                md = d
            if md <= 0.0:
                return md
    return md


def _ppe(lon, lat, lon1, lat1):
    a = lat1 - lat
    b = lon1 - lon
    return math.sqrt(a * a + b * b)


def point_bbox_distance(x, y, x1, y1, x2, y2):
    def border(x1_, y1_, x2_, y2_):
        if x1_ == x2_:
            return _ppe(x, y, x1_, y)
        if y1_ == y2_:
            return _ppe(x, y, x, y1_)
        return 5e-324
    if x <= x1:
        if y <= y1:
            return _ppe(x, y, x1, y1)
        if y >= y2:
            return _ppe(x, y, x1, y2)
        return border(x1, y1, x1, y2)
    if x >= x2:
        if y <= y1:
            return _ppe(x, y, x2, y1)
        if y >= y2:
            return _ppe(x, y, x2, y2)
        return border(x2, y1, x2, y2)
    if y <= y1:
        return border(x1, y1, x2, y1)
    if y >= y2:
        return border(x1, y2, x2, y2)
    return 0.0


def _close(ring):
    ring = [tuple(map(float, v)) for v in ring]
    return ring if ring[0] == ring[-1] else ring + [ring[0]]


def range_ppoly(grid, xs, ys, polys, r, approximate=False):
    polys = [[_close(rg) for rg in p] for p in polys]
    G, C = set(), set()
    bbs = []
    for p in polys:
        sx = [v[0] for v in p[0]]
        sy = [v[1] for v in p[0]]
        bb = (min(sx), min(sy), max(sx), max(sy))
        bbs.append(bb)
        x1, y1 = grid.cell(bb[0], bb[1])
        x2, y2 = grid.cell(bb[2], bb[3])
        ids = [cell_id(a, b) for a in range(x1, x2 + 1) for b in range(y1, y2 + 1)]
        Gp = set()
        for cid in ids:
            Gp |= g_set(grid, r, cid)
        G |= Gp
        Cp = set()
        for cid in ids:
            Cp |= c_set(grid, r, cid, G)
        C |= Cp
    out = []
    for i, (x, y) in enumerate(zip(xs, ys)):
        k = cell_id(*grid.cell(x, y))
        if k in G:
            out.append(i)
        elif k in C:
            for p, bb in zip(polys, bbs):
                d = point_bbox_distance(x, y, *bb) if approximate else point_polygon_distance(x, y, p)
                if d <= r:
                    out.append(i)
                    break
    return out


def knn_contract(grid, xs, ys, objs, qx, qy, r, k):
    cid = cell_id(*grid.cell(qx, qy))
    G = g_set(grid, r, cid)
    C = c_set(grid, r, cid, G)
    best = {}
    for i, (x, y, o) in enumerate(zip(xs, ys, objs)):
        key = cell_id(*grid.cell(x, y))
        if key not in G and key not in C:
            continue
        d = dist(qx, qy, x, y)
        if not d <= r:
            continue
        if o not in best or (d, i) < best[o]:
            best[o] = (d, i)
    lst = sorted((d, o, i) for o, (d, i) in best.items())
    return lst[:k]


def join_pp(ugrid, qgrid, oxs, oys, qxs, qys, r, approximate=False):
    if r == 0:
        rep_cells = lambda q: [cell_id(i, j) for i in range(qgrid.n) for j in range(qgrid.n)]  # noqa: E731
    else:
        c = qgrid.c_layers(r)
        if c <= 0:
            return None

        def rep_cells(q):
            px, py = parse_id(cell_id(*qgrid.cell(qxs[q], qys[q])))
            return [cell_id(i, j) for i in range(max(px - c, 0), min(px + c, qgrid.n - 1) + 1)
                    for j in range(max(py - c, 0), min(py + c, qgrid.n - 1) + 1)]
    buckets = {}
    for q in range(len(qxs)):
        for cid in rep_cells(q):
            buckets.setdefault(cid, []).append(q)
    out = []
    for p, (x, y) in enumerate(zip(oxs, oys)):
        for q in buckets.get(cell_id(*ugrid.cell(x, y)), ()):
            if approximate or dist(x, y, qxs[q], qys[q]) <= r:
                out.append((p, q))
    return out


def join_ppoly(ugrid, qgrid, xs, ys, polys, r, approximate=False):
    """PointPolygonJoinQuery.windowBased: polygon q replicated to its own G_q u C_q
    (getReplicatedPolygonQueryStream), point p joined on its gridID, kept if approximate or
    getDistance(p, q) <= r.  Returns sorted (point, polygon) pairs."""
    polys = [[_close(rg) for rg in p] for p in polys]
    buckets = {}
    for q, p in enumerate(polys):
        sx = [v[0] for v in p[0]]
        sy = [v[1] for v in p[0]]
        x1, y1 = qgrid.cell(min(sx), min(sy))
        x2, y2 = qgrid.cell(max(sx), max(sy))
        ids = [cell_id(a, b) for a in range(x1, x2 + 1) for b in range(y1, y2 + 1)]
        Gq = set()
        for cid in ids:
            Gq |= g_set(qgrid, r, cid)
        Cq = set()
        for cid in ids:
            Cq |= c_set(qgrid, r, cid, Gq)
        for k in Gq | Cq:
            buckets.setdefault(k, []).append(q)
    out = []
    for i, (x, y) in enumerate(zip(xs, ys)):
        for q in buckets.get(cell_id(*ugrid.cell(x, y)), ()):
            if approximate or point_polygon_distance(x, y, polys[q]) <= r:
                out.append((i, q))
    return sorted(out)
