"""Spatial operators -- mirrors of GeoFlink.spatialOperators.{range,knn,join} for one window.

The reference builds a Flink DAG per operator and evaluates each window inside a
WindowFunction.apply; here run() takes the window's points (a PointWindow, device SoA) and
evaluates that window on the GPU through the C ABI -- the body of apply() is what moved.

  PointPointRangeQuery.run(window, Set<Point>, r)     -- range/PointPointRangeQuery.java:37,111-187
  PointPolygonRangeQuery.run(window, Set<Polygon>, r) -- range/PointPolygonRangeQuery.java:31,134-205
  PointPointKNNQuery.run(window, Point, r, k)         -- knn/PointPointKNNQuery.java:33,132-201
  PointPointJoinQuery.run(ordinary, query, r)         -- join/PointPointJoinQuery.java:24,124-183
  PointPolygonJoinQuery.run(points, polygons, r)      -- join/PointPolygonJoinQuery.java:154-213

Errors follow the reference: unsupported query types raise ValueError ("Not yet support",
IllegalArgumentException), candidate layers <= 0 raise CandidateLayersError (System.exit(1)).
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
from dataclasses import dataclass
from enum import Enum

import numpy as np

from . import _lib
from .spatialIndices import UniformGrid
from .spatialObjects import Point, PointWindow, Polygon, PolygonSet


class QueryType(Enum):
    """QueryType.java:3-8"""
    RealTime = 0
    WindowBased = 1
    CountBased = 2
    RealTimeNaive = 3


class QueryConfiguration:
    """QueryConfiguration.java:5-57 (+ distanceMetric: JTS Coordinate.distance variant)."""

    def __init__(self, queryType: QueryType = None):
        self.queryType = queryType
        self.windowSize = 0
        self.slideStep = 0
        self.allowedLateness = 0
        self.approximateQuery = False
        self.distanceMetric = _lib.METRIC_SQRT

    def getQueryType(self): return self.queryType
    def setQueryType(self, t): self.queryType = t
    def getWindowSize(self): return self.windowSize
    def setWindowSize(self, v): self.windowSize = int(v)
    def getSlideStep(self): return self.slideStep
    def setSlideStep(self, v): self.slideStep = int(v)
    def getAllowedLateness(self): return self.allowedLateness
    def setAllowedLateness(self, v): self.allowedLateness = int(v)
    def isApproximateQuery(self): return self.approximateQuery
    def setApproximateQuery(self, v): self.approximateQuery = bool(v)


_SUPPORTED = (QueryType.RealTime, QueryType.WindowBased)


def _require_supported(conf: QueryConfiguration):
    # RealTime and WindowBased share the per-point semantics evaluated here (the RealTime
    # flatMap bodies equal the window apply bodies); the others throw in the reference too.
    if conf.getQueryType() not in _SUPPORTED:
        raise ValueError("Not yet support")


class _PlanCache:
    """Device plans of one operator, keyed by query CONTENTS (coordinates, polygon digest,
    radius, flags) and bounded: the least recently used plan beyond `limit` is destroyed, so a
    query stream (a new polygon set per window) does not leak one device plan per window."""

    def __init__(self, destroy_name: str, limit: int = 16):
        self._destroy_name = destroy_name
        self.limit = int(limit)
        self._d = OrderedDict()
        self._pinned = set()  # plans with state beyond their key (pipeline, capacity, a pane engine)

    def pin(self, plan):
        """Never evict `plan`: a plan with settings or pending pipelined work, or one a pane
        engine (gf_*_sliding) holds, lives until it is unpinned or the operator closes."""
        self._pinned.add(self._pv(plan))

    def unpin(self, plan):
        """The holder of a pin is done with it (a pane engine closed): the plan is an ordinary
        LRU entry again and is evicted if the cache is over its limit."""
        self._pinned.discard(self._pv(plan))
        self._evict(None)

    def get(self, key):
        plan = self._d.get(key)
        if plan is not None:
            self._d.move_to_end(key)
        return plan

    def put(self, key, plan):
        self._d[key] = plan
        self._evict(key)

    def _evict(self, keep):
        """Destroy least recently used unpinned plans beyond `limit`, never `keep` (the plan being
        inserted, which the caller is about to use): with `limit` pinned plans the cache simply
        grows past its limit until pins are released."""
        over = len(self._d) - self.limit
        if over <= 0:
            return
        victims = [k for k, p in self._d.items() if k != keep and self._pv(p) not in self._pinned][:over]
        for k in victims:
            self._destroy(self._d.pop(k))

    @staticmethod
    def _pv(plan):
        return plan.value if hasattr(plan, "value") else plan

    def _destroy(self, plan):
        if _lib._lib is not None:
            getattr(_lib._lib, self._destroy_name)(plan)

    def __len__(self):
        return len(self._d)

    def close(self):
        while self._d:
            _, p = self._d.popitem(last=False)
            self._destroy(p)
        self._pinned.clear()


class SpatialOperator:
    _destroy_name = "gf_range_plan_destroy"

    def __init__(self, conf: QueryConfiguration, index: UniformGrid):
        self.conf = conf
        self.index = index
        self._plans = _PlanCache(self._destroy_name)

    def getQueryConfiguration(self):
        return self.conf

    def getSpatialIndex(self):
        return self.index


# ----------------------------------------------------------------------------------------
# range
# ----------------------------------------------------------------------------------------
@dataclass
class RangeResult:
    """Selection bitmap of one window (bit i = point i emitted) plus counts.

    For approximate point-point queries with |Q| > 1 the reference emits candidate-cell
    points once per query point: `multi` marks those points (multiplicity |Q|)."""

    window: PointWindow
    bitmap: object          # torch int64 [(n+63)/64] (uint64 words)
    counts: object          # torch int64 [2]: points emitted, multiset size
    multi: object = None
    nq: int = 1
    ctx: object = None

    def count(self) -> int:
        return int(self.counts[0].item())

    def multiset_size(self) -> int:
        return int(self.counts[1].item())

    def indices(self) -> np.ndarray:
        """Ascending indices of emitted points (each once)."""
        return bitmap_indices(self.ctx, self.bitmap, self.window.n)

    def multiset_indices(self) -> np.ndarray:
        idx = self.indices().astype(np.int64)
        if self.multi is None or self.nq <= 1:
            return idx
        m = bitmap_indices(self.ctx, self.multi, self.window.n).astype(np.int64)
        return np.sort(np.concatenate([idx] + [m] * (self.nq - 1)), kind="stable")

    def points(self, uGrid=None):
        return [self.window.point(i, uGrid) for i in self.indices()]


def bitmap_indices(ctx, bitmap, n) -> np.ndarray:
    import torch

    cap = max(1, int(n))
    out = torch.empty(cap, dtype=torch.int32, device=bitmap.device)
    cnt = C.c_int64()
    st = _lib.lib().gf_bitmap_to_indices(ctx.handle, bitmap.data_ptr(), int(n), out.data_ptr(), cap, C.byref(cnt))
    _lib.check(st, ctx.handle, "gf_bitmap_to_indices")
    return out[: cnt.value].cpu().numpy().view(np.uint32)


class _RangeBase(SpatialOperator):
    def _evaluate(self, plan, window: PointWindow, nq: int) -> RangeResult:
        import torch

        ctx = _lib.context(window.x.device.index)
        n = window.n
        words = max(1, (n + 63) // 64)
        bitmap = torch.empty(words, dtype=torch.int64, device=window.x.device)
        multi = torch.empty(words, dtype=torch.int64, device=window.x.device) if nq > 1 else None
        counts = torch.zeros(2, dtype=torch.int64, device=window.x.device)
        pts = window.c_struct()
        st = _lib.lib().gf_range_run(plan, C.byref(pts), bitmap.data_ptr(),
                                     multi.data_ptr() if multi is not None else None, counts.data_ptr())
        _lib.check(st, ctx.handle, "gf_range_run")
        return RangeResult(window, bitmap, counts, multi, nq, ctx)

    def _plan(self, key, create):
        plan = self._plans.get(key)
        if plan is None:
            plan = create()
            self._plans.put(key, plan)
            tuning = getattr(self, "tuning", None)  # (scan_blocks, defer_mode): gf_range_plan_set_tuning
            if tuning is not None:
                _lib.check(_lib.lib().gf_range_plan_set_tuning(plan, int(tuning[0]), int(tuning[1])), None,
                           "gf_range_plan_set_tuning")
            lanes = getattr(self, "drain_lanes", None)  # testing: gf_range_plan_set_drain_lanes
            if lanes is not None:
                _lib.check(_lib.lib().gf_range_plan_set_drain_lanes(plan, int(lanes)), None,
                           "gf_range_plan_set_drain_lanes")
        return plan

    def __del__(self):
        plans = getattr(self, "_plans", None)
        if plans is not None:
            plans.close()


class PointPointRangeQuery(_RangeBase):
    """range/PointPointRangeQuery.java -- window-based point-point range query."""

    def run(self, window: PointWindow, queryPointSet, queryRadius: float) -> RangeResult:
        _require_supported(self.conf)
        qs = list(queryPointSet)
        ctx, plan = self.plan(window.x.device.index, qs, queryRadius)
        nq = len(qs) if self.conf.approximateQuery else 1
        return self._evaluate(plan, window, nq)

    def plan(self, device: int, queryPointSet, queryRadius: float):
        """(context, gf_range_plan) of this query on `device` (cached by query contents)."""
        _require_supported(self.conf)
        qs = list(queryPointSet)
        qx = np.array([q.x for q in qs], np.float64)
        qy = np.array([q.y for q in qs], np.float64)
        ctx = _lib.context(device)
        key = (ctx.device, tuple(qx.tolist()), tuple(qy.tolist()), float(queryRadius),
               bool(self.conf.approximateQuery), int(self.conf.distanceMetric))

        def create():
            h = C.c_void_p()
            st = _lib.lib().gf_range_pp_plan_create(ctx.handle, C.byref(self.index.c_grid), qx.ctypes.data,
                                                    qy.ctypes.data, len(qs), float(queryRadius),
                                                    int(self.conf.approximateQuery), int(self.conf.distanceMetric),
                                                    C.byref(h))
            _lib.check(st, ctx.handle, "gf_range_pp_plan_create")
            return h

        return ctx, self._plan(key, create)


class PointPolygonRangeQuery(_RangeBase):
    """range/PointPolygonRangeQuery.java -- window-based point-polygon range query."""

    def run(self, window: PointWindow, queryPolygonSet, queryRadius: float) -> RangeResult:
        _require_supported(self.conf)
        ctx, plan = self.plan(window.x.device.index, queryPolygonSet, queryRadius)
        return self._evaluate(plan, window, 1)

    def plan(self, device: int, queryPolygonSet, queryRadius: float):
        """(context, gf_range_plan) of this query on `device` (cached by query contents)."""
        _require_supported(self.conf)
        ps = PolygonSet(queryPolygonSet)
        ctx = _lib.context(device)
        key = (ctx.device, ps.digest(), float(queryRadius), bool(self.conf.approximateQuery),
               int(self.conf.distanceMetric))

        def create():
            cs = ps.c_struct()
            h = C.c_void_p()
            st = _lib.lib().gf_range_ppoly_plan_create(ctx.handle, C.byref(self.index.c_grid), C.byref(cs),
                                                       float(queryRadius), int(self.conf.approximateQuery),
                                                       int(self.conf.distanceMetric), C.byref(h))
            _lib.check(st, ctx.handle, "gf_range_ppoly_plan_create")
            return h

        return ctx, self._plan(key, create)


# ----------------------------------------------------------------------------------------
# kNN
# ----------------------------------------------------------------------------------------
@dataclass
class KNNResult:
    """Tuple3<winStart, winEnd, PriorityQueue<Tuple2<Point, Double>>> as sorted arrays:
    rank i = (objID[i], dist[i]), point index idx[i] in the window."""

    windowStart: int
    windowEnd: int
    objID: np.ndarray
    dist: np.ndarray
    idx: np.ndarray

    def __len__(self):
        return len(self.objID)

    def tuples(self):
        return list(zip(self.objID.tolist(), self.dist.tolist()))


def knn_record_bytes(k: int) -> int:
    return int(_lib.lib().gf_knn_result_bytes(int(k)))


def decode_knn_record(raw: bytes, k: int):
    """Decode a host copy of a device kNN record -> (status, objID, dist, idx)."""
    h = _lib.GfKnnHeader.from_buffer_copy(raw[: C.sizeof(_lib.GfKnnHeader)])
    off = C.sizeof(_lib.GfKnnHeader)
    d = np.frombuffer(raw, np.float64, k, off)
    o = np.frombuffer(raw, np.int64, k, off + 8 * k)
    i = np.frombuffer(raw, np.int64, k, off + 16 * k)
    return h.status, o[: h.n].copy(), d[: h.n].copy(), i[: h.n].copy()


class PinnedRecords:
    """A ring of kNN records in mapped pinned host memory (gf_pinned_alloc).  Pass
    `ptr(i)` as the record of enqueue(): the select kernel writes the record straight into
    host memory, so no copy kernel runs per window; read `raw(i)` after the stream syncs."""

    def __init__(self, count: int, k: int):
        self.k = int(k)
        self.count = int(count)
        self.bytes = knn_record_bytes(k)
        p = C.c_void_p()
        _lib.check(_lib.lib().gf_pinned_alloc(self.bytes * self.count, C.byref(p)), None, "gf_pinned_alloc")
        self._base = p.value
        self.view = np.ctypeslib.as_array((C.c_uint8 * (self.bytes * self.count)).from_address(self._base))
        self.view[:] = 0

    def ptr(self, i: int) -> int:
        return self._base + (i % self.count) * self.bytes

    def raw(self, i: int) -> bytes:
        j = i % self.count
        return self.view[j * self.bytes:(j + 1) * self.bytes].tobytes()

    def decode(self, i: int):
        return decode_knn_record(self.raw(i), self.k)

    def __del__(self):
        base = getattr(self, "_base", None)
        if base and _lib._lib is not None:
            self.view = None
            _lib._lib.gf_pinned_free(C.c_void_p(base))
            self._base = None


class PointPointKNNQuery(SpatialOperator):
    """knn/PointPointKNNQuery.java -- continuous kNN of one query point within radius r."""

    _destroy_name = "gf_knn_plan_destroy"

    def __init__(self, conf: QueryConfiguration, index: UniformGrid):
        super().__init__(conf, index)
        self._depth = {}  # plan handle -> pipeline depth (set_pipeline)

    @staticmethod
    def _pv(plan):
        return plan.value if hasattr(plan, "value") else plan

    def plan(self, window_device: int, queryPoint: Point, queryRadius: float, k: int):
        ctx = _lib.context(window_device)
        key = (ctx.device, queryPoint.x, queryPoint.y, float(queryRadius), int(k), int(self.conf.distanceMetric))
        plan = self._plans.get(key)
        if plan is None:
            h = C.c_void_p()
            st = _lib.lib().gf_knn_pp_plan_create(ctx.handle, C.byref(self.index.c_grid), float(queryPoint.x),
                                                  float(queryPoint.y), float(queryRadius), int(k),
                                                  int(self.conf.distanceMetric), C.byref(h))
            _lib.check(st, ctx.handle, "gf_knn_pp_plan_create")
            self._plans.put(key, h)
            plan = h
        return ctx, plan

    def run(self, window: PointWindow, queryPoint: Point, queryRadius: float, k: int) -> KNNResult:
        _require_supported(self.conf)
        if k is None or int(k) < 1:
            raise ValueError("k must be >= 1 (PriorityQueue initialCapacity < 1)")
        ctx, plan = self.plan(window.x.device.index, queryPoint, queryRadius, k)
        kk = int(k)
        oo = np.empty(kk, np.int64); od = np.empty(kk, np.float64); oi = np.empty(kk, np.int64)
        n = C.c_int32()
        pts = window.c_struct()
        st = _lib.lib().gf_knn_run(plan, C.byref(pts), oo.ctypes.data, od.ctypes.data, oi.ctypes.data, C.byref(n))
        _lib.check(st, ctx.handle, "gf_knn_run")
        m = n.value
        return KNNResult(window.start, window.end, oo[:m].copy(), od[:m].copy(), oi[:m].copy())

    def enqueue(self, window: PointWindow, queryPoint: Point, queryRadius: float, k: int, record):
        """Async: evaluate the window into a record -- a torch uint8 device tensor of
        knn_record_bytes(k), or an int address from PinnedRecords.ptr() (kernel writes the
        host record directly); pair with finish() once the record is on the host.  The window's
        tensors must stay alive until the record is complete (at depth >= 3 kernels on the plan's
        other streams read them, which torch's caching allocator does not track)."""
        ctx, plan = self.plan(window.x.device.index, queryPoint, queryRadius, k)
        pts = window.c_struct()
        addr = record if isinstance(record, int) else record.data_ptr()
        # depth >= 3 launches windows on the plan's other streams, which do not wait for the
        # context stream (torch's current stream, where this window's tensors were produced):
        # every enqueue orders those streams after it (gf_ctx_fork records one event), so a
        # window refilled in place on torch's stream is complete before any kernel reads it
        if self._depth.get(self._pv(plan), 1) >= 3:
            _lib.check(_lib.lib().gf_ctx_fork(ctx.handle), ctx.handle, "gf_ctx_fork")
        _lib.check(_lib.lib().gf_knn_enqueue(plan, C.byref(pts), C.c_void_p(addr)), ctx.handle, "gf_knn_enqueue")

    def finish(self, window: PointWindow, queryPoint: Point, queryRadius: float, k: int, raw: bytes) -> KNNResult:
        ctx, plan = self.plan(window.x.device.index, queryPoint, queryRadius, k)
        kk = int(k)
        oo = np.empty(kk, np.int64); od = np.empty(kk, np.float64); oi = np.empty(kk, np.int64)
        n = C.c_int32()
        buf = C.create_string_buffer(bytes(raw), len(raw))
        pts = window.c_struct()
        st = _lib.lib().gf_knn_decode(plan, C.byref(pts), buf, oo.ctypes.data, od.ctypes.data, oi.ctypes.data,
                                      C.byref(n))
        _lib.check(st, ctx.handle, "gf_knn_decode")
        m = n.value
        return KNNResult(window.start, window.end, oo[:m].copy(), od[:m].copy(), oi[:m].copy())

    def set_pipeline(self, window_device, queryPoint, queryRadius, k, depth: int):
        """depth 2: one fused launch per window; window i's record is written by the next
        enqueue (its select runs in block 0 of window i+1's scan) or by flush()."""
        ctx, plan = self.plan(window_device, queryPoint, queryRadius, k)
        _lib.check(_lib.lib().gf_knn_plan_set_pipeline(plan, int(depth)), ctx.handle, "set_pipeline")
        self._plans.pin(plan)  # its depth and pending records must survive the LRU
        self._depth[self._pv(plan)] = int(depth)

    def flush(self, window_device, queryPoint, queryRadius, k):
        ctx, plan = self.plan(window_device, queryPoint, queryRadius, k)
        _lib.check(_lib.lib().gf_knn_plan_flush(plan), ctx.handle, "flush")

    def set_capacity(self, window_device, queryPoint, queryRadius, k, cap):
        ctx, plan = self.plan(window_device, queryPoint, queryRadius, k)
        _lib.check(_lib.lib().gf_knn_plan_set_capacity(plan, int(cap)), ctx.handle, "set_capacity")
        self._plans.pin(plan)

    def __del__(self):
        plans = getattr(self, "_plans", None)
        if plans is not None:
            plans.close()


class PointPolygonKNNQuery(PointPointKNNQuery):
    """knn/PointPolygonKNNQuery.java -- continuous kNN of the window's points to one query
    polygon within r (JTS point-polygon distance, 0 inside; approximate: the bbox distance).
    Same run / enqueue / finish API as PointPointKNNQuery with a Polygon as the query."""

    def plan(self, window_device: int, queryPolygon: Polygon, queryRadius: float, k: int):
        ctx = _lib.context(window_device)
        ps = PolygonSet([queryPolygon])
        key = (ctx.device, ps.digest(), float(queryRadius), int(k), int(self.conf.distanceMetric),
               bool(self.conf.isApproximateQuery()))
        plan = self._plans.get(key)
        if plan is None:
            cs = ps.c_struct()
            h = C.c_void_p()
            st = _lib.lib().gf_knn_ppoly_plan_create(ctx.handle, C.byref(self.index.c_grid), C.byref(cs),
                                                     float(queryRadius), int(k), int(self.conf.isApproximateQuery()),
                                                     int(self.conf.distanceMetric), C.byref(h))
            _lib.check(st, ctx.handle, "gf_knn_ppoly_plan_create")
            self._plans.put(key, h)
            plan = h
        return ctx, plan


def knn_merge_host(k: int, lists):
    """Top-k distinct objIDs of several sorted (objID, dist, idx) lists -- the windowAll funnel
    (KNNQuery.java:213-272) across shards; host code of the library (no GPU needed)."""
    counts = np.array([len(l[0]) for l in lists], np.int32)
    o = np.ascontiguousarray(np.concatenate([np.asarray(l[0], np.int64) for l in lists]) if lists else
                             np.zeros(0, np.int64))
    d = np.ascontiguousarray(np.concatenate([np.asarray(l[1], np.float64) for l in lists]) if lists else
                             np.zeros(0, np.float64))
    i = np.ascontiguousarray(np.concatenate([np.asarray(l[2], np.int64) for l in lists]) if lists else
                             np.zeros(0, np.int64))
    oo = np.empty(k, np.int64); od = np.empty(k, np.float64); oi = np.empty(k, np.int64)
    n = C.c_int32()
    st = _lib.lib().gf_knn_merge_host(int(k), len(lists), counts.ctypes.data, o.ctypes.data, d.ctypes.data,
                                      i.ctypes.data, oo.ctypes.data, od.ctypes.data, oi.ctypes.data, C.byref(n))
    _lib.check(st, None, "gf_knn_merge_host")
    return oo[: n.value].copy(), od[: n.value].copy(), oi[: n.value].copy()


# ----------------------------------------------------------------------------------------
# join
# ----------------------------------------------------------------------------------------
class PointPointJoinQuery(SpatialOperator):
    """join/PointPointJoinQuery.java -- window-based point-point join.  index1 = uGrid
    (ordinary stream), index2 = qGrid (query stream, replicated to neighbour cells)."""

    def __init__(self, conf: QueryConfiguration, index1: UniformGrid, index2: UniformGrid = None):
        super().__init__(conf, index1)
        self.index2 = index2 if index2 is not None else index1

    def run(self, ordinaryWindow: PointWindow, queryWindow: PointWindow, queryRadius: float) -> np.ndarray:
        """Returns int64 [m, 2] pairs (ordinary index, query index), sorted."""
        import torch

        _require_supported(self.conf)
        ctx = _lib.context(ordinaryWindow.x.device.index)
        po, pq = ordinaryWindow.c_struct(), queryWindow.c_struct()
        cap = max(1024, 4 * (ordinaryWindow.n + queryWindow.n))
        for _ in range(2):
            pairs = torch.empty(2 * cap, dtype=torch.int32, device=ordinaryWindow.x.device)
            npairs = C.c_int64()
            st = _lib.lib().gf_join_pp(ctx.handle, C.byref(self.index.c_grid), C.byref(self.index2.c_grid),
                                       C.byref(po), C.byref(pq), float(queryRadius), int(self.conf.approximateQuery),
                                       int(self.conf.distanceMetric), pairs.data_ptr(), cap, C.byref(npairs))
            if st == _lib.GF_ERR_CAPACITY:
                cap = int(npairs.value)
                continue
            _lib.check(st, ctx.handle, "gf_join_pp")
            m = int(npairs.value)
            out = pairs[: 2 * m].cpu().numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
            order = np.lexsort((out[:, 1], out[:, 0]))
            return out[order]
        raise _lib.GeoFlinkError(_lib.GF_ERR_CAPACITY, "join output kept growing")


class PointPolygonJoinQuery(_RangeBase):
    """join/PointPolygonJoinQuery.java -- window-based join of a point stream with a polygon
    stream (PointPolygonJoinQuery.java:154-213; polygons replicated to their own guaranteed +
    candidate cells, JoinQuery.java:93-115).  index1 = uGrid (points), index2 = qGrid
    (polygons); the device path requires the two grids to be equal.  The replicated polygon
    side is a plan, cached by the polygons' contents (a static query set reuses it; a polygon
    stream's window with new geometry builds a new one, the cache keeps the 16 most recent)."""

    def __init__(self, conf: QueryConfiguration, index1: UniformGrid, index2: UniformGrid = None):
        super().__init__(conf, index1)
        self.index2 = index2 if index2 is not None else index1

    def run(self, pointWindow: PointWindow, queryPolygons, queryRadius: float) -> np.ndarray:
        """Returns int64 [m, 2] pairs (point index, polygon index), sorted."""
        import torch

        _require_supported(self.conf)
        ps = PolygonSet(queryPolygons)  # keeps the CSR arrays alive during the call
        ctx = _lib.context(pointWindow.x.device.index)
        key = (ctx.device, ps.digest(), float(queryRadius), bool(self.conf.approximateQuery),
               int(self.conf.distanceMetric))

        def create():
            cs = ps.c_struct()
            h = C.c_void_p()
            _lib.check(_lib.lib().gf_join_ppoly_plan_create(ctx.handle, C.byref(self.index2.c_grid), C.byref(cs),
                                                            float(queryRadius), int(self.conf.approximateQuery),
                                                            int(self.conf.distanceMetric), C.byref(h)),
                       ctx.handle, "gf_join_ppoly_plan_create")
            return h

        plan = self._plan(key, create)
        pts = pointWindow.c_struct()
        cap = max(1024, 2 * pointWindow.n)
        for _ in range(2):
            pairs = torch.empty(2 * cap, dtype=torch.int32, device=pointWindow.x.device)
            npairs = C.c_int64()
            st = _lib.lib().gf_join_ppoly_run(plan, C.byref(self.index.c_grid), C.byref(pts), pairs.data_ptr(), cap,
                                              C.byref(npairs))
            if st == _lib.GF_ERR_CAPACITY:
                cap = int(npairs.value)
                continue
            _lib.check(st, ctx.handle, "gf_join_ppoly_run")
            m = int(npairs.value)
            out = pairs[: 2 * m].cpu().numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
            order = np.lexsort((out[:, 1], out[:, 0]))
            return out[order]
        raise _lib.GeoFlinkError(_lib.GF_ERR_CAPACITY, "join output kept growing")


# ----------------------------------------------------------------------------------------
# cell assignment / bucketing (the ingest-side pieces of the path)
# ----------------------------------------------------------------------------------------
def assign_cells(window: PointWindow, grid: UniformGrid):
    """K1: HelperClass.assignGridCellID for every point -> (cx, cy) int32 torch tensors."""
    import torch

    ctx = _lib.context(window.x.device.index)
    n = window.n
    cx = torch.empty(max(n, 1), dtype=torch.int32, device=window.x.device)
    cy = torch.empty(max(n, 1), dtype=torch.int32, device=window.x.device)
    pts = window.c_struct()
    _lib.check(_lib.lib().gf_assign_cells(ctx.handle, C.byref(grid.c_grid), C.byref(pts), cx.data_ptr(),
                                          cy.data_ptr()), ctx.handle, "gf_assign_cells")
    return cx[:n], cy[:n]


def bucket_by_cell(window: PointWindow, grid: UniformGrid):
    """K2: keyBy(gridID) analogue -> (perm, cell_start) with bucket n*n = out-of-grid."""
    import torch

    ctx = _lib.context(window.x.device.index)
    n = window.n
    g = grid.getNumGridPartitions()
    perm = torch.empty(max(n, 1), dtype=torch.int32, device=window.x.device)
    start = torch.empty(g * g + 2, dtype=torch.int32, device=window.x.device)
    pts = window.c_struct()
    _lib.check(_lib.lib().gf_bucket_by_cell(ctx.handle, C.byref(grid.c_grid), C.byref(pts), perm.data_ptr(),
                                            start.data_ptr()), ctx.handle, "gf_bucket_by_cell")
    return perm[:n], start


def synthetic_uniform(seed: int, n: int, minX: float, maxX: float, minY: float, maxY: float):
    """java.util.Random(seed)-compatible uniform points (SyntheticGpsSource.java:23,40-41)."""
    x = np.empty(n, np.float64)
    y = np.empty(n, np.float64)
    _lib.check(_lib.lib().gf_synth_uniform(int(seed), int(n), float(minX), float(maxX), float(minY), float(maxY),
                                           x.ctypes.data, y.ctypes.data), None, "gf_synth_uniform")
    return x, y


def synthetic_clustered(seed: int, n: int, minX: float, maxX: float, minY: float, maxY: float, centers=None,
                        n_centers: int = 8, sigma: float = 0.01, frac: float = 0.8):
    """The clustered variant of the synthetic source: a fraction `frac`
    of the points from Gaussian hot spots N(centre, sigma^2) (sigma in degrees), the rest
    uniform; `centers` (list of (x, y)) come first, the remaining of `n_centers` are uniform in
    the bounds.  Points falling outside the bounds are drawn again, so every point is inside.
    numpy PCG64(seed): deterministic, host-side (input generation, not the evaluated path)."""
    rng = np.random.default_rng(seed)
    cs = [tuple(c) for c in (centers or [])][:n_centers]
    while len(cs) < n_centers:
        cs.append((rng.uniform(minX, maxX), rng.uniform(minY, maxY)))
    cx = np.array([c[0] for c in cs], np.float64)
    cy = np.array([c[1] for c in cs], np.float64)
    x = np.empty(n, np.float64)
    y = np.empty(n, np.float64)
    todo = np.arange(n)
    while len(todo):
        m = len(todo)
        hot = rng.random(m) < frac
        k = rng.integers(0, len(cs), m)
        xv = np.where(hot, cx[k] + sigma * rng.standard_normal(m), rng.uniform(minX, maxX, m))
        yv = np.where(hot, cy[k] + sigma * rng.standard_normal(m), rng.uniform(minY, maxY, m))
        ok = (xv >= minX) & (xv < maxX) & (yv >= minY) & (yv < maxY)
        x[todo[ok]] = xv[ok]
        y[todo[ok]] = yv[ok]
        todo = todo[~ok]
    return x, y


__all__ = [
    "synthetic_clustered", "QueryType", "QueryConfiguration", "PointPointRangeQuery", "PointPolygonRangeQuery", "PointPointKNNQuery",
    "PointPointJoinQuery", "PointPolygonJoinQuery", "RangeResult", "KNNResult", "knn_merge_host", "assign_cells", "bucket_by_cell",
    "synthetic_uniform", "Point", "Polygon", "PointWindow", "knn_record_bytes", "decode_knn_record",
]
