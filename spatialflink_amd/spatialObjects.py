"""Spatial objects -- mirrors of GeoFlink.spatialObjects.{Point, Polygon} plus the SoA window
batch that crosses the C ABI at each window trigger.

A PointWindow is the device-resident struct-of-arrays form of a window's Iterable<Point>:
x, y (float64, 16-B aligned), objID and timeStampMillisec (int64), as torch CUDA tensors.
objID strings are carried as their int64 decimal value.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _lib
from .spatialIndices import UniformGrid, generateCellIDStr


class Point:
    """Point(String objID, double x, double y, long timeStampMillisec, UniformGrid) -- Point.java:91-100"""

    __slots__ = ("objID", "x", "y", "timeStampMillisec", "gridID")

    def __init__(self, objID, x: float, y: float, timeStampMillisec: int = 0, uGrid: Optional[UniformGrid] = None,
                 gridID: Optional[str] = None):
        self.objID = objID
        self.x = float(x)
        self.y = float(y)
        self.timeStampMillisec = int(timeStampMillisec)
        if gridID is not None:
            self.gridID = gridID
        elif uGrid is not None:
            self.gridID = uGrid.assignGridCellID(self.x, self.y)  # Point.java:98
        else:
            self.gridID = ""

    def __repr__(self):
        return f"Point(objID={self.objID}, x={self.x!r}, y={self.y!r}, ts={self.timeStampMillisec}, gridID={self.gridID})"


def _ring_area(ring):
    a = 0.0
    for (x1, y1), (x2, y2) in zip(ring[:-1], ring[1:]):
        a += x1 * y2 - x2 * y1
    return abs(a) / 2.0


class Polygon:
    """Polygon(List<List<Coordinate>> coordinates, UniformGrid) -- Polygon.java:52-66.

    Rings are closed if needed (createPolygon, :147-165); with several rings the largest-area
    ring becomes the shell (createPolygonArray ordering, :115-145).  boundingBox is the shell
    envelope (HelperClass.getBoundingBox :76-80); gridIDsSet = every cell under the bbox
    (HelperClass.assignGridCellID(bBox) :123-143)."""

    def __init__(self, coordinates, uGrid: Optional[UniformGrid] = None, objID=None, timeStampMillisec: int = 0):
        if len(coordinates) < 1 or len(coordinates[0]) <= 3:
            raise ValueError("Polygon needs a ring with more than 3 coordinates (Polygon.java:53)")
        rings = []
        for ring in coordinates:
            ring = [(float(x), float(y)) for x, y in ring]
            if 0 < len(ring) < 4:
                ring = ring + [ring[0]] * 4
            if ring[0] != ring[-1]:
                ring.append(ring[0])
            rings.append(ring)
        if len(rings) > 1:
            ordered = []
            for r in rings:  # createPolygonArray: keep descending area
                if not ordered or _ring_area(ordered[-1]) >= _ring_area(r):
                    ordered.append(r)
                else:
                    for i in range(len(ordered)):
                        if _ring_area(ordered[i]) <= _ring_area(r):
                            ordered.insert(i, r)
                            break
            rings = ordered
        self.rings = rings
        self.objID = objID
        self.timeStampMillisec = int(timeStampMillisec)
        sx = [v[0] for v in rings[0]]
        sy = [v[1] for v in rings[0]]
        self.boundingBox = ((min(sx), min(sy)), (max(sx), max(sy)))
        self.gridID = ""
        self.gridIDsSet = set()
        if uGrid is not None:
            (x1, y1), (x2, y2) = self.boundingBox
            a1, b1 = uGrid.cellOf(x1, y1)
            a2, b2 = uGrid.cellOf(x2, y2)
            self.gridIDsSet = {generateCellIDStr(a, b) for a in range(a1, a2 + 1) for b in range(b1, b2 + 1)}

    def __repr__(self):
        return f"Polygon(rings={len(self.rings)}, bbox={self.boundingBox})"


class PolygonSet:
    """Host CSR of a polygon set for the C ABI (gf_polygons)."""

    def __init__(self, polygons):
        self.polygons = list(polygons)
        ring_off, vert_off, vx, vy = [0], [0], [], []
        for p in self.polygons:
            for ring in p.rings:
                vx += [v[0] for v in ring]
                vy += [v[1] for v in ring]
                vert_off.append(len(vx))
            ring_off.append(len(vert_off) - 1)
        self.ring_off = np.asarray(ring_off, np.int32)
        self.vert_off = np.asarray(vert_off, np.int32)
        self.vx = np.asarray(vx, np.float64)
        self.vy = np.asarray(vy, np.float64)

    def c_struct(self) -> _lib.GfPolygons:
        return _lib.GfPolygons(len(self.polygons), self.ring_off.ctypes.data, self.vert_off.ctypes.data,
                               self.vx.ctypes.data, self.vy.ctypes.data)

    def digest(self) -> bytes:
        """Content key of the set (ring layout + every vertex bit pattern): device plans are
        cached by it, so a new polygon list with the same geometry reuses a plan and any other
        geometry never does (object ids are recycled by CPython, contents are not)."""
        import hashlib

        h = hashlib.blake2b(digest_size=20)
        for a in (self.ring_off, self.vert_off, self.vx, self.vy):
            h.update(np.int64(a.size).tobytes())
            h.update(np.ascontiguousarray(a).tobytes())
        return h.digest()


@dataclass
class PointWindow:
    """One window's points as device SoA (torch CUDA tensors)."""

    x: "object"
    y: "object"
    objID: "object"
    timeStampMillisec: "object"
    start: int = 0
    end: int = 0
    extra: dict = field(default_factory=dict)

    @property
    def n(self) -> int:
        return int(self.x.numel())

    @classmethod
    def from_numpy(cls, x, y, objID=None, ts=None, device=None, start=0, end=0):
        import torch

        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        n = len(x)
        objID = np.arange(n, dtype=np.int64) if objID is None else objID
        ts = np.zeros(n, dtype=np.int64) if ts is None else ts
        t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a, dtype=dt)).to(dev)  # noqa: E731
        return cls(t(x, np.float64), t(y, np.float64), t(objID, np.int64), t(ts, np.int64), start, end)

    @classmethod
    def from_points(cls, points, device=None, start=0, end=0):
        x = np.array([p.x for p in points], np.float64)
        y = np.array([p.y for p in points], np.float64)
        o = np.array([int(p.objID) for p in points], np.int64)
        ts = np.array([p.timeStampMillisec for p in points], np.int64)
        return cls.from_numpy(x, y, o, ts, device, start, end)

    def c_struct(self) -> _lib.GfPoints:
        for t in (self.x, self.y):
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("PointWindow tensors must be contiguous CUDA tensors")
        return _lib.GfPoints(self.x.data_ptr(), self.y.data_ptr(), self.objID.data_ptr(),
                             self.timeStampMillisec.data_ptr(), self.n)

    def point(self, i: int, uGrid: Optional[UniformGrid] = None) -> Point:
        i = int(i)
        return Point(str(int(self.objID[i])), float(self.x[i]), float(self.y[i]), int(self.timeStampMillisec[i]),
                     uGrid)
