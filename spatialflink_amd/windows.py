"""Sliding windows -- Flink's SlidingProcessingTimeWindows as used by the reference operators
(PointPointKNNQuery.java:158,198-200; PointPointRangeQuery.java:149), evaluated pane by pane.

The reference re-evaluates every window from scratch, so each point is processed size/slide
times.  Here the stream is cut into panes of gcd(size, slide) ms (Flink window assignment with
offset 0: pane p holds timestamps [p*pane, (p+1)*pane)); each pane is evaluated once on the
GPU and a window's result is assembled from its panes:

  kNN    -- the device pane engine (gf_knn_sliding_*): one fused scan/select launch per pane
            into a record ring, one merge launch per window (top-k-distinct of a union = the
            merge of the parts' top-k-distinct lists, so it equals evaluating the window whole);
  range  -- the per-pane selection bitmaps (range results are per point: a window's hits are
            the concatenation of its panes' hits).

Batches arrive in timestamp order (processing-time ingestion) and are cut into panes on the
device (gf_pane_bounds).  Windows fire only if they hold a point (Flink keeps no state for
empty windows).  Window timestamps are in ms; the reference's Time.seconds(windowSize) is
windowSize * 1000.
"""
from __future__ import annotations

import ctypes as C
import math
from collections import OrderedDict

import numpy as np

from . import _lib
from .spatialObjects import Point, PointWindow
from .spatialOperators import (KNNResult, PinnedRecords, PointPointKNNQuery, QueryConfiguration,
                               _require_supported, bitmap_indices)


class SlidingWindows:
    """SlidingProcessingTimeWindows.of(size, slide) geometry (offset 0)."""

    def __init__(self, size_ms: int, slide_ms: int):
        if size_ms <= 0 or slide_ms <= 0:
            raise ValueError("window size and slide must be > 0")
        self.size = int(size_ms)
        self.slide = int(slide_ms)
        self.pane = math.gcd(self.size, self.slide)
        self.panes_per_window = self.size // self.pane
        self.panes_per_slide = self.slide // self.pane

    @classmethod
    def from_conf(cls, conf: QueryConfiguration):
        """QueryConfiguration windowSize / slideStep are seconds (Time.seconds(...))."""
        return cls(int(conf.getWindowSize()) * 1000, int(conf.getSlideStep() or conf.getWindowSize()) * 1000)

    def assign_windows(self, ts: int):
        """Window starts containing timestamp ts (Flink SlidingProcessingTimeWindows.assignWindows:
        lastStart = TimeWindow.getWindowStartWithOffset(ts, 0, slide), then every slide back
        while start > ts - size)."""
        last = ts - (ts + self.slide) % self.slide
        out = []
        s = last
        while s > ts - self.size:
            out.append(s)
            s -= self.slide
        return out

    def pane_of(self, ts):
        return np.floor_divide(np.asarray(ts, np.int64), self.pane)

    def closes(self, pane_index: int) -> bool:
        """Windows start at multiples of slide: pane p ends one iff (p+1)*pane - size is one."""
        return (pane_index + 1 - self.panes_per_window) % self.panes_per_slide == 0

    def window_of_last_pane(self, pane_index: int):
        end = (pane_index + 1) * self.pane
        return end - self.size, end


def pane_bounds(batch: PointWindow, pane_ms: int, first_pane: int, npanes: int) -> np.ndarray:
    """Device split of a time-ordered batch into panes first_pane .. first_pane+npanes-1:
    returns int64[npanes + 1] slice bounds (gf_pane_bounds)."""
    import torch

    ctx = _lib.context(batch.x.device.index)
    out = torch.empty(npanes + 1, dtype=torch.int64, device=batch.x.device)
    _lib.check(_lib.lib().gf_pane_bounds(ctx.handle, batch.timeStampMillisec.data_ptr(), batch.n, int(pane_ms),
                                         int(first_pane), int(npanes), out.data_ptr()), ctx.handle, "gf_pane_bounds")
    return out.cpu().numpy()


def _slice(w: PointWindow, lo: int, hi: int) -> PointWindow:
    """Device view of [lo, hi); the scans load x, y as 16-B pairs, so a pane starting at an
    odd element is copied to a fresh (aligned) buffer."""
    x, y = w.x[lo:hi], w.y[lo:hi]
    if (x.data_ptr() | y.data_ptr()) & 15:
        x, y = x.clone(), y.clone()
    return PointWindow(x, y, w.objID[lo:hi], w.timeStampMillisec[lo:hi])


class _PaneStream:
    """Cuts time-ordered batches into consecutive panes; the slices are device views."""

    def __init__(self, geo: SlidingWindows):
        self.geo = geo
        self.next_pane = None   # index of the pane being filled
        self.parts = []         # slices of the pane being filled (it can span batches)

    def feed(self, batch: PointWindow):
        """Yield (pane_index, PointWindow or None when empty) for every pane this batch completes."""
        if batch.n == 0:
            return
        ts0 = int(batch.timeStampMillisec[0].item())
        ts1 = int(batch.timeStampMillisec[-1].item())
        p0, p1 = ts0 // self.geo.pane, ts1 // self.geo.pane
        if self.next_pane is None:
            self.next_pane = p0
        if p0 < self.next_pane:
            raise ValueError("batch timestamps precede the current pane (late data is not supported)")
        b = pane_bounds(batch, self.geo.pane, self.next_pane, p1 - self.next_pane + 1)
        for j in range(len(b) - 1):
            lo, hi = int(b[j]), int(b[j + 1])
            if hi > lo:
                self.parts.append(_slice(batch, lo, hi))
            if self.next_pane + j < p1:  # a later pane has started: this one is complete
                yield self.next_pane + j, self._take()
        self.next_pane = p1

    def _take(self):
        import torch

        parts, self.parts = self.parts, []
        if not parts:
            return None
        if len(parts) == 1:
            return parts[0]
        cat = lambda f: torch.cat([getattr(p, f) for p in parts])  # noqa: E731
        return PointWindow(cat("x"), cat("y"), cat("objID"), cat("timeStampMillisec"))

    def close(self):
        """The pane being filled, if any (end of stream)."""
        if self.next_pane is None or not self.parts:
            return None
        p = self.next_pane
        self.next_pane += 1
        return p, self._take()


class SlidingKNNQuery:
    """Continuous sliding-window kNN -- PointPointKNNQuery.windowBased with
    SlidingProcessingTimeWindows.of(size, slide) (PointPointKNNQuery.java:132-201).

    push(batch) consumes time-ordered points; results() returns the KNNResult of every window
    that has fired so far (windowStart, windowEnd, objID/dist sorted by (dist, objID), idx =
    position of the point in its window, i.e. in the window's panes concatenated in time
    order)."""

    def __init__(self, conf: QueryConfiguration, grid, queryPoint: Point, queryRadius: float, k: int,
                 size_ms: int = None, slide_ms: int = None, device: int = 0, pipeline: int = 2):
        _require_supported(conf)
        if k is None or int(k) < 1:
            raise ValueError("k must be >= 1 (PriorityQueue initialCapacity < 1)")
        self.geo = SlidingWindows(size_ms, slide_ms) if size_ms else SlidingWindows.from_conf(conf)
        self.k = int(k)
        self.op = PointPointKNNQuery(conf, grid)
        self.ctx, self.plan = self.op.plan(device, queryPoint, queryRadius, k)
        self.op._plans.pin(self.plan)  # the pane engine holds it
        self.depth = int(pipeline)  # k > 256: the select is not fused, records complete in stream order
        _lib.check(_lib.lib().gf_knn_plan_set_pipeline(self.plan, self.depth), self.ctx.handle, "set_pipeline")
        h = C.c_void_p()
        _lib.check(_lib.lib().gf_knn_sliding_create(self.plan, self.geo.size, self.geo.slide, C.byref(h)),
                   self.ctx.handle, "gf_knn_sliding_create")
        self.handle = h
        ring = C.c_int32()
        _lib.check(_lib.lib().gf_knn_sliding_geometry(h, None, None, None, C.byref(ring)), self.ctx.handle, "geometry")
        self.ring = ring.value
        self.records = PinnedRecords(self.ring, self.k)
        self.panes = OrderedDict()   # pane index -> (PointWindow, stream position); the engine borrows them
        self.pos = 0
        self.last_pane = None
        self.closed = []             # (window_end, record slot, first pane)
        self.nclosed = 0
        self.pending = False         # depth 2: the newest closed window's record is not written yet
        self.ready = []              # decoded KNNResults not yet returned by results()
        self.stream = _PaneStream(self.geo)

    # -- panes ---------------------------------------------------------------------------
    def push_pane(self, pane_index: int, pane: PointWindow):
        """Push one pane (consecutive indices; gaps are filled with empty panes)."""
        if self.last_pane is not None:
            for p in range(self.last_pane + 1, pane_index):
                self._push_one(p, None)
        self._push_one(pane_index, pane)

    def _push_one(self, p, pane):
        empty = pane is None or pane.n == 0
        cs = _lib.GfPoints(None, None, None, None, 0) if empty else pane.c_struct()
        slot = self.nclosed % self.ring
        closed, end = C.c_int32(), C.c_int64()
        st = _lib.lib().gf_knn_sliding_push(self.handle, int(p), C.byref(cs), C.c_void_p(self.records.ptr(slot)),
                                            C.byref(closed), C.byref(end))
        _lib.check(st, self.ctx.handle, "gf_knn_sliding_push")
        self.panes[p] = (None if empty else pane, self.pos)
        self.pos += 0 if empty else pane.n
        while len(self.panes) > self.ring:
            self.panes.popitem(last=False)
        self.last_pane = p
        self.pending = False
        if closed.value:
            self.closed.append((end.value, slot, p - self.geo.panes_per_window + 1))
            self.nclosed += 1
            self.pending = self.depth == 2 and not empty
        # a flagged record is re-evaluated from its panes, which the engine keeps for `ring`
        # panes only: decode before the oldest undecoded window's panes leave the ring
        if self.closed and p - self.closed[0][2] >= self.ring - 2:
            self._collect()

    def push(self, batch: PointWindow):
        for p, pane in self.stream.feed(batch):
            self.push_pane(p, pane)

    def flush(self):
        """End of input (Flink's final watermark): push the pane being filled, then empty panes
        until every window holding a point has fired, and complete every pending record."""
        last = self.stream.close()
        if last is not None:
            self.push_pane(*last)
        if self.last_pane is not None:
            g = self.geo
            last_start = (self.last_pane * g.pane // g.slide) * g.slide
            for p in range(self.last_pane + 1, (last_start + g.size) // g.pane):
                self._push_one(p, None)
        _lib.check(_lib.lib().gf_knn_sliding_flush(self.handle), self.ctx.handle, "gf_knn_sliding_flush")
        self.pending = False

    def results(self):
        """KNNResults of the windows fired so far whose records are complete (syncs)."""
        self._collect()
        out, self.ready = self.ready, []
        return out

    def _collect(self):
        import torch

        torch.cuda.synchronize(self.ctx.device)
        ready = self.closed[:-1] if self.pending else self.closed
        self.closed = self.closed[len(ready):]
        for end, slot, first in ready:
            base = self.panes[first][1] if first in self.panes else self._base_of(first)
            oo = np.empty(self.k, np.int64); od = np.empty(self.k, np.float64); oi = np.empty(self.k, np.int64)
            n = C.c_int32()
            buf = C.create_string_buffer(self.records.raw(slot), self.records.bytes)
            st = _lib.lib().gf_knn_sliding_decode(self.handle, int(end), buf, oo.ctypes.data, od.ctypes.data,
                                                  oi.ctypes.data, C.byref(n))
            _lib.check(st, self.ctx.handle, "gf_knn_sliding_decode")
            m = n.value
            self.ready.append(KNNResult(end - self.geo.size, end, oo[:m].copy(), od[:m].copy(), oi[:m] - base))

    def _base_of(self, first):
        for q, (_, pos) in self.panes.items():
            if q >= first:
                return pos
        return self.pos

    def close(self):
        """Destroy the pane engine and release its pin on the plan."""
        h = getattr(self, "handle", None)
        if h and _lib._lib is not None:
            _lib._lib.gf_knn_sliding_destroy(h)
            self.handle = None
            self.op._plans.unpin(self.plan)

    def __del__(self):
        self.close()


class SlidingRangeQuery:
    """Sliding-window range query (PointPointRangeQuery / PointPolygonRangeQuery with
    SlidingProcessingTimeWindows, PointPointRangeQuery.java:149-186) on the device pane engine
    (gf_range_sliding_*): each pane is evaluated once, a closed window's hits (positions within
    the window, ascending) are assembled on the device from its panes' index lists, and
    results() reads every fired window after one stream sync."""

    def __init__(self, op, queries, queryRadius: float, size_ms: int, slide_ms: int):
        self.op = op
        self.queries = queries
        self.r = queryRadius
        self.geo = SlidingWindows(size_ms, slide_ms)
        self.stream = _PaneStream(self.geo)
        self.handle = None
        self.ctx = None
        self.last_pane = None
        self.fired = []              # (start, end, device idx, device count)

    def _engine(self, device):
        import torch

        if self.handle is None:
            self.ctx, plan = self.op.plan(device, self.queries, self.r)
            self.op._plans.pin(plan)
            self.plan = plan
            h = C.c_void_p()
            _lib.check(_lib.lib().gf_range_sliding_create(plan, self.geo.size, self.geo.slide, C.byref(h)),
                       self.ctx.handle, "gf_range_sliding_create")
            self.handle = h
            self._spare = torch.empty(1, dtype=torch.int32, device=f"cuda:{self.ctx.device}")
        return self.handle

    def _pane(self, p, pane):
        if self.last_pane is not None:
            for q in range(self.last_pane + 1, p):
                self._one(q, None)
        self._one(p, pane)

    def _one(self, p, pane):
        import torch

        if self.handle is None:
            if pane is None:
                return  # nothing before the first pane with points
            self._engine(pane.x.device.index)
        empty = pane is None or pane.n == 0
        cs = _lib.GfPoints(None, None, None, None, 0) if empty else pane.c_struct()
        closed, end, wn = C.c_int32(), C.c_int64(), C.c_int64()
        dev = f"cuda:{self.ctx.device}"
        idx, cnt = self._spare, torch.zeros(1, dtype=torch.int64, device=dev)
        while True:  # the window's index buffer: sized from the window's points on a capacity miss
            st = _lib.lib().gf_range_sliding_push(self.handle, int(p), C.byref(cs), idx.data_ptr(), idx.numel(),
                                                  cnt.data_ptr(), C.byref(closed), C.byref(end), C.byref(wn))
            if st != _lib.GF_ERR_CAPACITY:
                break
            idx = torch.empty(int(wn.value), dtype=torch.int32, device=dev)
        _lib.check(st, self.ctx.handle, "gf_range_sliding_push")
        self._spare = torch.empty(1, dtype=torch.int32, device=dev) if closed.value else idx
        self.last_pane = p
        if closed.value:
            self.fired.append((end.value - self.geo.size, end.value, idx, cnt))

    def push(self, batch: PointWindow):
        for p, pane in self.stream.feed(batch):
            self._pane(p, pane)

    def flush(self):
        """End of input (Flink's final watermark): the pane being filled, then empty panes until
        every window holding a point has fired -- as SlidingKNNQuery.flush."""
        last = self.stream.close()
        if last is not None:
            self._pane(*last)
        if self.last_pane is not None:
            g = self.geo
            last_start = (self.last_pane * g.pane // g.slide) * g.slide
            for p in range(self.last_pane + 1, (last_start + g.size) // g.pane):
                self._one(p, None)

    def results(self):
        """(windowStart, windowEnd, hits) of every window fired so far; hits = ascending
        positions within the window (its panes concatenated in time order)."""
        if not self.fired:
            return []
        fired, self.fired = self.fired, []
        self.ctx.synchronize()
        out = []
        for s0, e, idx, cnt in fired:
            m = int(cnt.item())
            out.append((s0, e, idx[:m].cpu().numpy().view(np.uint32).astype(np.int64)))
        return out

    def close(self):
        """Destroy the pane engine and release its pin on the operator's plan."""
        if getattr(self, "handle", None) is not None and _lib._lib is not None:
            _lib.lib().gf_range_sliding_destroy(self.handle)
            self.handle = None
            self.op._plans.unpin(self.plan)

    def __del__(self):
        self.close()
