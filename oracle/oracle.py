"""ctypes + numpy harness for the C oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  It is the checker: the product path (spatialflink_amd + libgeoflink_hip.so)
never imports it.  Parity status of the oracle: "parity unpinned" (see
oracle/geoflink_oracle.h and DESIGN.md).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# GF_ORACLE_LIB: another build of the same sources (`make asan`: -fsanitize=address,undefined)
_SO = os.environ.get("GF_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")

METRIC_SQRT = 0
METRIC_HYPOT = 1
ERR_LAYERS = -5
ERR_NPE = -6


class OrcGrid(C.Structure):
    _fields_ = [("n", C.c_int32), ("minX", C.c_double), ("maxX", C.c_double),
                ("minY", C.c_double), ("maxY", C.c_double), ("cellLength", C.c_double)]


class OrcPolygons(C.Structure):
    _fields_ = [("npoly", C.c_int32), ("ring_off", C.c_void_p), ("vert_off", C.c_void_p),
                ("vx", C.c_void_p), ("vy", C.c_void_p)]


def build():
    if not os.environ.get("GF_ORACLE_LIB"):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        P = C.c_void_p
        d, i32, i64 = C.c_double, C.c_int32, C.c_int64
        L.orc_grid_make.argtypes = [i32, d, d, d, d, C.POINTER(OrcGrid)]
        L.orc_jint.argtypes = [d]; L.orc_jint.restype = i32
        L.orc_cell_id.argtypes = [i32, i32, C.c_char_p]
        L.orc_parse_cell_id.argtypes = [C.c_char_p, C.POINTER(i32), C.POINTER(i32)]
        L.orc_assign_cells.argtypes = [C.POINTER(OrcGrid), i64, P, P, P, P]
        L.orc_guaranteed_layers.argtypes = [C.POINTER(OrcGrid), d]; L.orc_guaranteed_layers.restype = i32
        L.orc_candidate_layers.argtypes = [C.POINTER(OrcGrid), d]; L.orc_candidate_layers.restype = i32
        L.orc_distance.argtypes = [d, d, d, d, C.c_int]; L.orc_distance.restype = d
        L.orc_hypot.argtypes = [d, d]; L.orc_hypot.restype = d
        L.orc_gc_sets_point.argtypes = [C.POINTER(OrcGrid), d, i32, i32, P, i64, C.POINTER(i64), P, i64, C.POINTER(i64)]
        L.orc_range_pp.argtypes = [C.POINTER(OrcGrid), i64, P, P, i32, P, P, d, C.c_int, C.c_int, P, i64]
        L.orc_range_pp.restype = i64
        L.orc_point_polygon_distance.argtypes = [d, d, C.POINTER(OrcPolygons), i32, C.c_int]
        L.orc_point_polygon_distance.restype = d
        L.orc_point_bbox_distance.argtypes = [d, d, d, d, d, d]; L.orc_point_bbox_distance.restype = d
        L.orc_range_ppoly.argtypes = [C.POINTER(OrcGrid), i64, P, P, C.POINTER(OrcPolygons), d, C.c_int, C.c_int, P, i64]
        L.orc_range_ppoly.restype = i64
        for fn in (L.orc_knn_contract, L.orc_knn_reference):
            fn.argtypes = [C.POINTER(OrcGrid), i64, P, P, P, d, d, d, i32, C.c_int, P, P, P]
            fn.restype = i32
        for fn in (L.orc_knn_reference_mt, L.orc_knn_scan_omp):
            fn.argtypes = [C.POINTER(OrcGrid), i64, P, P, P, d, d, d, i32, C.c_int, C.c_int, P, P, P]
            fn.restype = i32
        L.orc_join_pp.argtypes = [C.POINTER(OrcGrid), C.POINTER(OrcGrid), i64, P, P, i64, P, P, d, C.c_int, C.c_int, P, i64]
        L.orc_join_pp.restype = i64
        L.orc_join_ppoly.argtypes = [C.POINTER(OrcGrid), C.POINTER(OrcGrid), i64, P, P, C.POINTER(OrcPolygons), d,
                                     C.c_int, C.c_int, P, i64]
        L.orc_join_ppoly.restype = i64
        L.orc_join_ppoly_mt.argtypes = [C.POINTER(OrcGrid), C.POINTER(OrcGrid), i64, P, P, C.POINTER(OrcPolygons), d,
                                        C.c_int, C.c_int, C.c_int, P, i64]
        L.orc_join_ppoly_mt.restype = i64
        L.orc_generate_query_polygons.argtypes = [i32, d, d, d, d, P, P, i32]
        L.orc_generate_query_polygons.restype = i32
        L.orc_java_random_points.argtypes = [i64, i64, d, d, d, d, P, P]
        L.orc_knn_ppoly_contract.argtypes = [C.POINTER(OrcGrid), i64, P, P, P, C.POINTER(OrcPolygons), d, i32,
                                             C.c_int, C.c_int, P, P, P]
        L.orc_knn_ppoly_contract.restype = i32
        L.orc_knn_ppoly_mt.argtypes = [C.POINTER(OrcGrid), i64, P, P, P, C.POINTER(OrcPolygons), d, i32,
                                       C.c_int, C.c_int, C.c_int, P, P, P]
        L.orc_knn_ppoly_mt.restype = i32
        L.orc_csv_parse.argtypes = [C.c_char_p, i64, C.c_char, P, P, P, C.c_char_p, i64, P, C.POINTER(i64), P, i64,
                                    C.POINTER(i64), C.POINTER(i32)]
        L.orc_csv_parse.restype = i64
        # multi-core baselines (bench cpu_baseline lines)
        L.orc_range_pp_mt.argtypes = [C.POINTER(OrcGrid), i64, P, P, i32, P, P, d, C.c_int, C.c_int, C.c_int, P, i64]
        L.orc_range_pp_mt.restype = i64
        L.orc_range_pp_omp.argtypes = L.orc_range_pp_mt.argtypes
        L.orc_range_pp_omp.restype = i64
        L.orc_range_ppoly_mt.argtypes = [C.POINTER(OrcGrid), i64, P, P, C.POINTER(OrcPolygons), d, C.c_int, C.c_int,
                                         C.c_int, P, i64]
        L.orc_range_ppoly_mt.restype = i64
        L.orc_range_ppoly_omp.argtypes = L.orc_range_ppoly_mt.argtypes
        L.orc_range_ppoly_omp.restype = i64
        L.orc_join_pp_mt.argtypes = [C.POINTER(OrcGrid), C.POINTER(OrcGrid), i64, P, P, i64, P, P, d, C.c_int, C.c_int,
                                     C.c_int, P, i64]
        L.orc_join_pp_mt.restype = i64
        L.orc_join_pp_omp.argtypes = [C.POINTER(OrcGrid), i64, P, P, i64, P, P, d, C.c_int, C.c_int, P, i64]
        L.orc_join_pp_omp.restype = i64
        L.orc_join_pp_omp_digest.argtypes = [C.POINTER(OrcGrid), i64, P, P, i64, P, P, d, C.c_int, C.c_int, P]
        L.orc_join_pp_omp_digest.restype = i64
        L.orc_csv_parse_mt.argtypes = [C.c_char_p, i64, C.c_char, P, P, P, P, i64, C.c_int, C.POINTER(i64),
                                       C.POINTER(i32)]
        L.orc_csv_parse_mt.restype = i64
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def grid(n, minX, maxX, minY, maxY):
    g = OrcGrid()
    rc = lib().orc_grid_make(int(n), float(minX), float(maxX), float(minY), float(maxY), C.byref(g))
    assert rc == 0
    return g


def jint(v):
    return lib().orc_jint(float(v))


def cell_id(cx, cy):
    buf = C.create_string_buffer(32)
    lib().orc_cell_id(int(cx), int(cy), buf)
    return buf.value.decode()


def parse_cell_id(s):
    a, b = C.c_int32(), C.c_int32()
    lib().orc_parse_cell_id(s.encode(), C.byref(a), C.byref(b))
    return a.value, b.value


def assign_cells(g, x, y):
    x, y = _f64(x), _f64(y)
    cx = np.empty(len(x), np.int32)
    cy = np.empty(len(x), np.int32)
    lib().orc_assign_cells(C.byref(g), len(x), _p(x), _p(y), _p(cx), _p(cy))
    return cx, cy


def layers(g, r):
    return lib().orc_guaranteed_layers(C.byref(g), float(r)), lib().orc_candidate_layers(C.byref(g), float(r))


def distance(x1, y1, x2, y2, metric=METRIC_SQRT):
    return lib().orc_distance(float(x1), float(y1), float(x2), float(y2), int(metric))


def hypot(a, b):
    return lib().orc_hypot(float(a), float(b))


def gc_sets_point(g, r, qcx, qcy):
    nG, nC = C.c_int64(), C.c_int64()
    lib().orc_gc_sets_point(C.byref(g), float(r), int(qcx), int(qcy), None, 0, C.byref(nG), None, 0, C.byref(nC))
    gc = np.empty((max(nG.value, 1), 2), np.int32)
    cc = np.empty((max(nC.value, 1), 2), np.int32)
    lib().orc_gc_sets_point(C.byref(g), float(r), int(qcx), int(qcy), _p(gc), nG.value, C.byref(nG), _p(cc), nC.value, C.byref(nC))
    gs = {tuple(map(int, v)) for v in gc[: nG.value]}
    cs = {tuple(map(int, v)) for v in cc[: nC.value]}
    return gs, cs


def range_pp(g, x, y, qx, qy, r, approximate=False, metric=METRIC_SQRT):
    x, y, qx, qy = _f64(x), _f64(y), _f64(np.atleast_1d(qx)), _f64(np.atleast_1d(qy))
    cap = max(1024, len(x))
    while True:
        out = np.empty(cap, np.int64)
        cnt = lib().orc_range_pp(C.byref(g), len(x), _p(x), _p(y), len(qx), _p(qx), _p(qy), float(r),
                                 int(approximate), int(metric), _p(out), cap)
        if cnt <= cap:
            return out[:cnt]
        cap = cnt


class Polygons:
    """CSR polygon set for the oracle: list of polygons, each a list of closed rings."""

    def __init__(self, polys):
        ring_off, vert_off, vx, vy = [0], [0], [], []
        for poly in polys:
            for ring in poly:
                ring = [tuple(map(float, v)) for v in ring]
                if ring[0] != ring[-1]:
                    ring.append(ring[0])
                vx += [v[0] for v in ring]
                vy += [v[1] for v in ring]
                vert_off.append(len(vx))
            ring_off.append(len(vert_off) - 1)
        self.ring_off = np.array(ring_off, np.int32)
        self.vert_off = np.array(vert_off, np.int32)
        self.vx = np.array(vx, np.float64)
        self.vy = np.array(vy, np.float64)
        self.c = OrcPolygons(len(polys), _p(self.ring_off).value, _p(self.vert_off).value,
                             _p(self.vx).value, _p(self.vy).value)


def point_polygon_distance(px, py, P: Polygons, p, metric=METRIC_SQRT):
    return lib().orc_point_polygon_distance(float(px), float(py), C.byref(P.c), int(p), int(metric))


def point_bbox_distance(px, py, x1, y1, x2, y2):
    return lib().orc_point_bbox_distance(*map(float, (px, py, x1, y1, x2, y2)))


def range_ppoly(g, x, y, P: Polygons, r, approximate=False, metric=METRIC_SQRT):
    x, y = _f64(x), _f64(y)
    cap = max(1024, len(x))
    out = np.empty(cap, np.int64)
    cnt = lib().orc_range_ppoly(C.byref(g), len(x), _p(x), _p(y), C.byref(P.c), float(r),
                                int(approximate), int(metric), _p(out), cap)
    assert cnt <= cap
    return out[:cnt]


def knn(g, x, y, objID, qx, qy, r, k, metric=METRIC_SQRT, reference_shaped=False):
    """Returns (status, objID[n], dist[n], idx[n]); contract output is sorted by (d, objID)."""
    x, y = _f64(x), _f64(y)
    objID = np.ascontiguousarray(objID, dtype=np.int64)
    kk = max(int(k), 1)
    oo = np.empty(kk, np.int64); od = np.empty(kk, np.float64); oi = np.empty(kk, np.int64)
    fn = lib().orc_knn_reference if reference_shaped else lib().orc_knn_contract
    n = fn(C.byref(g), len(x), _p(x), _p(y), _p(objID), float(qx), float(qy), float(r), int(k),
           int(metric), _p(oo), _p(od), _p(oi))
    if n < 0:
        return n, None, None, None
    return 0, oo[:n], od[:n], oi[:n]


def knn_mt(g, x, y, objID, qx, qy, r, k, nthreads, metric=METRIC_SQRT, optimized=False):
    """CPU baselines on nthreads host threads: the reference-shaped evaluator shaped as Flink's
    parallel operator (orc_knn_reference_mt, = knn(reference_shaped=True)) or the optimised
    OpenMP scan (orc_knn_scan_omp, = knn()).  Returns (status, objID, dist, idx)."""
    x, y = _f64(x), _f64(y)
    objID = np.ascontiguousarray(objID, dtype=np.int64)
    kk = max(int(k), 1)
    oo = np.empty(kk, np.int64); od = np.empty(kk, np.float64); oi = np.empty(kk, np.int64)
    fn = lib().orc_knn_scan_omp if optimized else lib().orc_knn_reference_mt
    n = fn(C.byref(g), len(x), _p(x), _p(y), _p(objID), float(qx), float(qy), float(r), int(k), int(metric),
           int(nthreads), _p(oo), _p(od), _p(oi))
    if n < 0:
        return n, None, None, None
    return 0, oo[:n], od[:n], oi[:n]


def host_cpu():
    """(nproc, lscpu model name) of this host."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return os.cpu_count() or 1, model


def join_pp(ugrid, qgrid, ox, oy, qx, qy, r, approximate=False, metric=METRIC_SQRT):
    """Returns (status, pairs[m,2]) with status < 0 for the reference's System.exit(1)."""
    ox, oy, qx, qy = _f64(ox), _f64(oy), _f64(qx), _f64(qy)
    cap = 1 << 16
    while True:
        out = np.empty(2 * cap, np.int64)
        cnt = lib().orc_join_pp(C.byref(ugrid), C.byref(qgrid), len(ox), _p(ox), _p(oy), len(qx), _p(qx),
                                _p(qy), float(r), int(approximate), int(metric), _p(out), cap)
        if cnt < 0:
            return int(cnt), None
        if cnt <= cap:
            return 0, out[: 2 * cnt].reshape(-1, 2)
        cap = int(cnt)


def _grow(fn, cap, width):
    while True:
        out = np.empty(width * max(cap, 1), np.int64)
        cnt = fn(out, max(cap, 1))
        if cnt < 0:
            raise ValueError(f"oracle baseline: status {cnt}")
        if cnt <= max(cap, 1):
            return out[: width * cnt].reshape(-1, width) if width > 1 else out[:cnt]
        cap = int(cnt)


def range_pp_mt(g, x, y, qx, qy, r, nthreads, approximate=False, metric=METRIC_SQRT, optimized=False):
    """orc_range_pp_mt (reference-shaped, Flink parallelism nthreads) or orc_range_pp_omp
    (optimised OpenMP): ascending indices, = range_pp."""
    x, y, qx, qy = _f64(x), _f64(y), _f64(np.atleast_1d(qx)), _f64(np.atleast_1d(qy))
    fn = lib().orc_range_pp_omp if optimized else lib().orc_range_pp_mt
    return _grow(lambda out, cap: fn(C.byref(g), len(x), _p(x), _p(y), len(qx), _p(qx), _p(qy), float(r),
                                     int(approximate), int(metric), int(nthreads), _p(out), cap), len(x), 1)


def range_ppoly_mt(g, x, y, P: "Polygons", r, nthreads, approximate=False, metric=METRIC_SQRT, optimized=False):
    x, y = _f64(x), _f64(y)
    fn = lib().orc_range_ppoly_omp if optimized else lib().orc_range_ppoly_mt
    return _grow(lambda out, cap: fn(C.byref(g), len(x), _p(x), _p(y), C.byref(P.c), float(r), int(approximate),
                                     int(metric), int(nthreads), _p(out), cap), len(x), 1)


def join_pp_mt(ugrid, qgrid, ox, oy, qx, qy, r, nthreads, metric=METRIC_SQRT, optimized=False):
    """Sorted pairs[m, 2]: orc_join_pp_mt (reference-shaped) or orc_join_pp_omp (optimised; one
    grid, exact, r > 0)."""
    ox, oy, qx, qy = _f64(ox), _f64(oy), _f64(qx), _f64(qy)
    if optimized:
        return _grow(lambda out, cap: lib().orc_join_pp_omp(C.byref(ugrid), len(ox), _p(ox), _p(oy), len(qx), _p(qx),
                                                            _p(qy), float(r), int(metric), int(nthreads), _p(out), cap),
                     1 << 16, 2)
    return _grow(lambda out, cap: lib().orc_join_pp_mt(C.byref(ugrid), C.byref(qgrid), len(ox), _p(ox), _p(oy), len(qx),
                                                       _p(qx), _p(qy), float(r), 0, int(metric), int(nthreads), _p(out),
                                                       cap), 1 << 16, 2)


def pair_digest(pairs) -> int:
    """Order-independent digest of (p, q) pairs: sum mod 2^64 of fmix64(p << 32 | q) (numpy, the
    oracle's orc_join_pp_omp_digest on the host side of a comparison)."""
    k = (np.asarray(pairs, np.int64).reshape(-1, 2).astype(np.uint64) * np.array([1 << 32, 1], np.uint64)).sum(axis=1)
    with np.errstate(over="ignore"):
        k ^= k >> np.uint64(33); k *= np.uint64(0xff51afd7ed558ccd); k ^= k >> np.uint64(33)
        k *= np.uint64(0xc4ceb9fe1a85ec53); k ^= k >> np.uint64(33)
        return int(k.sum(dtype=np.uint64))


def join_pp_digest(ugrid, ox, oy, qx, qy, r, nthreads, metric=METRIC_SQRT):
    """(pair count, pair_digest) of the optimised OpenMP join, no pair stored (windows with
    billions of pairs)."""
    ox, oy, qx, qy = _f64(ox), _f64(oy), _f64(qx), _f64(qy)
    dg = np.zeros(1, np.uint64)
    cnt = lib().orc_join_pp_omp_digest(C.byref(ugrid), len(ox), _p(ox), _p(oy), len(qx), _p(qx), _p(qy), float(r),
                                       int(metric), int(nthreads), _p(dg))
    if cnt < 0:
        raise ValueError(f"oracle join digest: status {cnt}")
    return int(cnt), int(dg[0])


def csv_parse_mt(text: bytes, delim: str, want, nthreads):
    """orc_csv_parse on nthreads parts of the chunk (a Flink map with that parallelism) ->
    (x, y, ts, bad_line, bad_kind)."""
    n = text.count(b"\n") + (0 if text.endswith(b"\n") or not text else 1)
    w = np.asarray(want, np.int32)
    x = np.zeros(n); y = np.zeros(n); t = np.zeros(n, np.int64)
    bl, bk = C.c_int64(), C.c_int32()
    lib().orc_csv_parse_mt(text, len(text), delim.encode(), _p(w), _p(x), _p(y), _p(t), n, int(nthreads),
                           C.byref(bl), C.byref(bk))
    return x, y, t, bl.value, bk.value


def join_ppoly(ugrid, qgrid, ox, oy, P: Polygons, r, approximate=False, metric=METRIC_SQRT):
    """Point-polygon window join (orc_join_ppoly): pairs[m, 2] = (point index, polygon index)."""
    ox, oy = _f64(ox), _f64(oy)
    cap = 1 << 16
    while True:
        out = np.empty(2 * cap, np.int64)
        cnt = lib().orc_join_ppoly(C.byref(ugrid), C.byref(qgrid), len(ox), _p(ox), _p(oy), C.byref(P.c), float(r),
                                   int(approximate), int(metric), _p(out), cap)
        if cnt <= cap:
            return out[: 2 * cnt].reshape(-1, 2)
        cap = int(cnt)


def join_ppoly_mt(ugrid, qgrid, ox, oy, P: "Polygons", r, nthreads, approximate=False, metric=METRIC_SQRT):
    """orc_join_ppoly_mt: the point-polygon join with Flink parallelism nthreads (the polygon side
    replicated once, the points in nthreads parts); sorted pairs[m, 2]."""
    ox, oy = _f64(ox), _f64(oy)
    return _grow(lambda out, cap: lib().orc_join_ppoly_mt(C.byref(ugrid), C.byref(qgrid), len(ox), _p(ox), _p(oy),
                                                          C.byref(P.c), float(r), int(approximate), int(metric),
                                                          int(nthreads), _p(out), cap), 1 << 16, 2)


def generate_query_polygons(num, minX, minY, maxX, maxY):
    cap = num + 256
    vx = np.empty(5 * cap); vy = np.empty(5 * cap)
    cnt = lib().orc_generate_query_polygons(int(num), float(minX), float(minY), float(maxX), float(maxY),
                                            _p(vx), _p(vy), cap)
    assert cnt <= cap
    return [[list(zip(vx[5 * i:5 * i + 5].tolist(), vy[5 * i:5 * i + 5].tolist()))] for i in range(cnt)]


def java_random_points(seed, n, minX, maxX, minY, maxY):
    x = np.empty(n); y = np.empty(n)
    lib().orc_java_random_points(int(seed), int(n), float(minX), float(maxX), float(minY), float(maxY), _p(x), _p(y))
    return x, y


def csv_parse(text: bytes, delim: str, want):
    """Deserialization.CSVTSVToTSpatial.map per line -> (x, y, objID Strings as a list of bytes,
    ts, bad_line, bad_kind)."""
    w = np.asarray(want, np.int32)
    bl, bk, ol = C.c_int64(), C.c_int32(), C.c_int64()
    n = lib().orc_csv_parse(text, len(text), delim.encode(), _p(w), None, None, None, 0, None, C.byref(ol), None, 0,
                            C.byref(bl), C.byref(bk))
    x = np.zeros(n); y = np.zeros(n); t = np.zeros(n, np.int64); off = np.zeros(n + 1, np.int64)
    ob = C.create_string_buffer(max(1, ol.value))
    lib().orc_csv_parse(text, len(text), delim.encode(), _p(w), _p(x), _p(y), ob, ol.value, _p(off), C.byref(ol), _p(t),
                        n, C.byref(bl), C.byref(bk))
    raw = ob.raw
    o = [raw[off[i]:off[i + 1]] for i in range(n)]
    return x, y, o, t, bl.value, bk.value


# ---------------------------------------------------------------------------------------------
# GeoJSON point ingest -- Deserialization.GeoJSONToTSpatial.map (Deserialization.java:149-211),
# restated over Python's json module (a JSON parser independent of the device scanner).  A line is
# the map's input ObjectNode: the Kafka record {"key": .., "value": ..} (JSONKeyValue-
# DeserializationSchema); value_lines: the record's value itself.  Per line:
#   Jackson reads the record: strict JSON (json.loads with NaN / Infinity refused, as Jackson's
#     defaults do; UTF-8 checked structurally, as Jackson's UTF-8 reader does) -> else kind 3;
#   V = record.get("value") (last duplicate); missing / not an object -> kind 3 (the map's NPE);
#   geometry = readGeoJSON(V.toString()) -- jts-io-common 1.18.0 GeoJsonReader (pom.xml:100-104,
#     absent from the reference tree; its published algorithm): V.type "Point" -> V.coordinates;
#     on failure, and for "Feature" (createFeature reads the same V.geometry) or a missing /
#     non-string / unknown type, the catch branch (:136-141, :172-178):
#     readGeoJSON(V.get("geometry").toString()) must be a Point, else the line fails;
#   time: dateFormat null -> Long.parseLong(String.valueOf(node)) (:190; a non-integer node throws
#         NumberFormatException), else dateFormat.parse(node.textValue()).getTime() (:187; a
#         ParseException leaves time 0, :193);
#   objID: node.toString().replaceAll("\"", "") (:197) -- a string's content, an integer's digits,
#          true / false / null as text; absent properties / objID -> null.
# Kinds as gf_geojson_parse: 1 NumberFormatException / ClassCastException of an ordinate, 2 outside
# the restated subset (include/geoflink_hip.h: non-Point geometries, FeatureCollection, < 2 or a
# non-number third ordinate, a number json-simple cannot read back anywhere on the line -- a float
# overflowing to Infinity or an integer outside long --, nesting > 256, escapes in taken strings or
# in member names of a looked-up object, non-integer objIDs, dates before 1583), 3 malformed /
# missing value or geometry, 4 empty line.
# ---------------------------------------------------------------------------------------------
_GEO_OTHER = {"LineString", "Polygon", "MultiPoint", "MultiLineString", "MultiPolygon", "GeometryCollection"}
_GEO_MAX_DEPTH = 256


def _jdate(v: str, tz_off_min: int):
    import calendar
    import re

    m = re.match(r"(\d+)-(\d+)-(\d+) (\d+):(\d+):(\d+)", v)
    if not m:
        return 0, 0                       # ParseException: time stays 0
    f = [int(g) for g in m.groups()]
    if any(len(g) >= 10 for g in m.groups()):  # int overflow territory of the lenient calendar
        return None, 2
    y = f[0] + (f[1] - 1) // 12           # SimpleDateFormat is lenient: fields roll over
    mo = (f[1] - 1) % 12 + 1
    if y < 1 or y > 9999:
        return None, 2
    secs = calendar.timegm((y, mo, 1, 0, 0, 0)) + (f[2] - 1) * 86400 + f[3] * 3600 + f[4] * 60 + f[5]
    if secs < -12219292800:               # before 1582-10-15: Java's Julian calendar
        return None, 2
    return secs * 1000 - tz_off_min * 60000, 0


class _JStr(str):
    """A decoded JSON string that remembers whether its source text held an escape."""
    escaped = False


class _JObj(dict):
    """A JSON object (last duplicate wins, Jackson ObjectNode) that remembers whether one of its
    member names was written with an escape."""
    esc_keys = False


def _too_deep(line: bytes) -> bool:
    """Nesting deeper than _GEO_MAX_DEPTH (brackets outside strings), on any input."""
    if line.count(b"{") + line.count(b"[") <= _GEO_MAX_DEPTH:
        return False
    d, st, i = 0, False, 0
    while i < len(line):
        c = line[i]
        if st:
            if c == 0x5C:
                i += 1
            elif c == 0x22:
                st = False
        elif c == 0x22:
            st = True
        elif c in (0x7B, 0x5B):
            d += 1
            if d > _GEO_MAX_DEPTH:
                return True
        elif c in (0x7D, 0x5D):
            d -= 1
        i += 1
    return False


def _utf8_structural(line: bytes) -> bool:
    """Jackson's UTF-8 reader: a lead byte 110xxxxx / 1110xxxx / 11110xxx takes 1 / 2 / 3 bytes
    10xxxxxx; no overlong / surrogate / range checks."""
    i, n = 0, len(line)
    while i < n:
        c = line[i]
        if c < 0x80:
            i += 1
            continue
        k = 1 if c & 0xE0 == 0xC0 else 2 if c & 0xF0 == 0xE0 else 3 if c & 0xF8 == 0xF0 else -1
        if k < 0 or i + k >= n:
            return False
        for j in range(1, k + 1):
            if line[i + j] & 0xC0 != 0x80:
                return False
        i += k + 1
    return True


def _json_decoder(escapes: bool, poison: list):
    """json's decoder, strict, with NaN / Infinity refused (Jackson), numbers json-simple could not
    read back flagged (poison[0]) and objects as _JObj; with escapes, the pure-Python scanner with
    strings tagged by escape use (the device reports a taken string or a looked-up object's member
    name written with an escape as unsupported)."""
    import json
    import json.scanner

    def pint(t):
        v = int(t)
        if not -(1 << 63) <= v < (1 << 63):
            poison[0] = True
        return v

    def pfloat(t):
        v = float(t)
        if math.isinf(v):
            poison[0] = True
        return v

    def pconst(t):
        raise ValueError(f"{t}: not JSON (Jackson's defaults refuse it)")

    def pairs(kv):
        d = _JObj(kv)
        d.esc_keys = any(getattr(k, "escaped", False) for k, _ in kv)
        return d

    dec = json.JSONDecoder(parse_int=pint, parse_float=pfloat, parse_constant=pconst, object_pairs_hook=pairs)
    if escapes:
        dec.parse_string = _tagged_scanstring
        dec.scan_once = json.scanner.py_make_scanner(dec)
    return dec


def _tagged_scanstring(s, end, strict=True):
    import json.decoder

    v, e = json.decoder.py_scanstring(s, end, strict)
    r = _JStr(v)
    r.escaped = "\\" in s[end:e]
    return r, e


class _Unsupported(Exception):
    pass


def _num(v):
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _point(c):
    """GeoJsonReader.createPoint's coordinates -> ("ok", x, y) / ("fail", kind) / ("unsup",)."""
    if not isinstance(c, list):
        return ("fail", 3)
    for i, v in enumerate(c[:3]):
        if not _num(v):
            return ("fail", 1) if i < 2 else ("unsup",)
    if len(c) < 2:
        return ("unsup",)
    x, y = float(c[0]), float(c[1])  # an int is Jackson's IntNode / LongNode: (double) of the long
    return ("ok", x, y)


def _gtype(obj, get):
    t = get(obj, "type")
    if not isinstance(t, str):
        return None
    if getattr(t, "escaped", False):
        raise _Unsupported()
    return t


def _geojson_line(line: bytes, prop_obj, prop_ts, date_fmt, tz_off_min, value_lines=False):
    if line.endswith(b"\r"):
        line = line[:-1]
    if not line:
        return None, 4
    if _too_deep(line):
        return None, 2
    if not _utf8_structural(line):
        return None, 3
    poison = [False]
    try:
        text = line.decode("utf-8", "surrogateescape")
        if b"\\" in line:  # member names go through json.decoder's module-level scanstring: tag them too
            import json.decoder as jd

            saved = jd.scanstring
            jd.scanstring = _tagged_scanstring
            try:
                d = _json_decoder(True, poison).decode(text)
            finally:
                jd.scanstring = saved
        else:
            d = _json_decoder(False, poison).decode(text)
    except ValueError:
        return None, 3
    if not isinstance(d, dict):
        return None, 3
    if poison[0]:
        return None, 2

    def get(obj, name):  # ObjectNode.get on an object the map looks a member up in
        if obj.esc_keys:
            raise _Unsupported()
        return obj.get(name)

    try:
        V = d if value_lines else get(d, "value")
        if not isinstance(V, dict):
            return None, 3
        xy = None
        tv = _gtype(V, get)
        if tv in _GEO_OTHER or tv == "FeatureCollection":
            return None, 2
        if tv == "Point":                      # readGeoJSON(value.toString())
            r = _point(get(V, "coordinates"))
            if r[0] == "unsup":
                return None, 2
            if r[0] == "ok":
                xy = r[1:]
        if xy is None:                         # the catch branch: readGeoJSON(value.get("geometry"))
            G = get(V, "geometry")
            if not isinstance(G, dict):
                return None, 3
            tg = _gtype(G, get)
            if tg is None or tg not in _GEO_OTHER | {"Point", "Feature", "FeatureCollection"}:
                return None, 3
            if tg != "Point":
                return None, 2
            r = _point(get(G, "coordinates"))
            if r[0] != "ok":
                return None, (2 if r[0] == "unsup" else r[1])
            xy = r[1:]
        x, y = xy
        ts, obj = 0, None
        props = get(V, "properties")
        if isinstance(props, dict) and (prop_ts is not None or prop_obj is not None):
            if props.esc_keys:
                raise _Unsupported()
            if prop_ts is not None and prop_ts in props:
                v = props[prop_ts]
                if date_fmt == 0:
                    if not (isinstance(v, int) and not isinstance(v, bool)) or not -(1 << 63) <= v < (1 << 63):
                        return None, 1
                    ts = v
                else:
                    if not isinstance(v, str):
                        return None, 1
                    if getattr(v, "escaped", False):  # the string is written with an escape
                        return None, 2
                    t, k = _jdate(v, tz_off_min)
                    if k:
                        return None, k
                    ts = t
            if prop_obj is not None and prop_obj in props:
                v = props[prop_obj]
                if isinstance(v, bool):
                    obj = b"true" if v else b"false"
                elif v is None:
                    obj = b"null"
                elif isinstance(v, int):
                    obj = str(v).encode()
                elif isinstance(v, str):
                    if getattr(v, "escaped", False):
                        return None, 2
                    obj = v.encode("utf-8", "surrogateescape")
                else:
                    return None, 2
    except _Unsupported:
        return None, 2
    return (x, y, ts, obj), 0


def geojson_parse(text: bytes, prop_obj=None, prop_ts=None, date_fmt=0, tz_off_min=0, value_lines=False):
    """GeoJSONToTSpatial.map per line -> (x, y, objID Strings as bytes or None, ts, bad_line,
    bad_kind); bad lines contribute zeros."""
    lines = text.split(b"\n")
    if lines and lines[-1] == b"" and text.endswith(b"\n"):
        lines = lines[:-1]
    n = len(lines)
    x = np.zeros(n); y = np.zeros(n); t = np.zeros(n, np.int64); o = [None] * n
    bad_line, bad_kind = -1, 0
    for i, ln in enumerate(lines):
        r, k = _geojson_line(ln, prop_obj, prop_ts, date_fmt, tz_off_min, value_lines)
        if k:
            if bad_line < 0:
                bad_line, bad_kind = i, k
            continue
        x[i], y[i], t[i], o[i] = r
    return x, y, o, t, bad_line, bad_kind


def knn_ppoly_mt(g, x, y, objID, P: "Polygons", r, k, nthreads, approximate=False, metric=METRIC_SQRT):
    """orc_knn_ppoly_mt: knn_ppoly with Flink parallelism nthreads (identical output)."""
    x, y, objID = _f64(x), _f64(y), np.ascontiguousarray(objID, np.int64)
    oo = np.zeros(k, np.int64); od = np.zeros(k); oi = np.zeros(k, np.int64)
    m = lib().orc_knn_ppoly_mt(C.byref(g), len(x), _p(x), _p(y), _p(objID), C.byref(P.c), float(r), int(k),
                               int(approximate), int(metric), int(nthreads), _p(oo), _p(od), _p(oi))
    if m < 0:
        raise ValueError(f"orc_knn_ppoly_mt: {m}")
    return m, oo[:m], od[:m], oi[:m]


def knn_ppoly(g, x, y, objID, P: "Polygons", r, k, approximate=False, metric=METRIC_SQRT):
    """PointPolygonKNNQuery (one query polygon) -> (n, objID, dist, idx), build contract."""
    x, y, objID = _f64(x), _f64(y), np.ascontiguousarray(objID, np.int64)
    oo = np.zeros(k, np.int64); od = np.zeros(k); oi = np.zeros(k, np.int64)
    m = lib().orc_knn_ppoly_contract(C.byref(g), len(x), _p(x), _p(y), _p(objID), C.byref(P.c), float(r), int(k),
                                     int(approximate), int(metric), _p(oo), _p(od), _p(oi))
    if m < 0:
        raise ValueError(f"orc_knn_ppoly_contract: {m}")
    return m, oo[:m], od[:m], oi[:m]
