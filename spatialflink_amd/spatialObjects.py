"""Spatial objects -- mirrors of GeoFlink.spatialObjects.{Point, Polygon} plus the SoA window
batch that crosses the C ABI at each window trigger.

A PointWindow is the device-resident struct-of-arrays form of a window's Iterable<Point>:
x, y (float64, 16-B aligned), objID and timeStampMillisec (int64), as torch CUDA tensors.
objID Strings (Point.objID) are carried as int64 keys (include/geoflink_hip.h "objID keys"):
a canonical decimal String is its value, any other String its id in an ObjIdDict.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _lib
from .spatialIndices import UniformGrid, generateCellIDStr


class ObjIdDict:
    """gf_objid_dict: String objIDs <-> int64 keys.  ObjIdDict.default(device) is the device
    context's dictionary, the one the CSV ingest uses; keys of one dictionary are equal iff
    their Strings are."""

    _defaults = {}

    def __init__(self, device: int = 0, handle=None, owned=True):
        self.device = int(device)
        self.ctx = _lib.context(self.device)
        if handle is None:
            h = C.c_void_p()
            _lib.check(_lib.lib().gf_objid_dict_create(self.ctx.handle, C.byref(h)), self.ctx.handle,
                       "gf_objid_dict_create")
            handle = h
        self.handle = handle
        self.owned = owned

    @classmethod
    def default(cls, device: int = 0) -> "ObjIdDict":
        ctx = _lib.context(int(device))
        key = id(ctx)
        d = cls._defaults.get(key)
        if d is None:
            h = C.c_void_p()
            _lib.check(_lib.lib().gf_ctx_objid_dict(ctx.handle, C.byref(h)), ctx.handle, "gf_ctx_objid_dict")
            d = cls(device, h, owned=False)
            cls._defaults[key] = d
        return d

    def size(self) -> int:
        n = C.c_int64()
        _lib.check(_lib.lib().gf_objid_dict_size(self.handle, C.byref(n)), None, "gf_objid_dict_size")
        return n.value

    def intern(self, objids) -> np.ndarray:
        """keys of Strings (str or bytes; str is UTF-8 encoded) -> int64[n]"""
        bs = [o.encode() if isinstance(o, str) else bytes(o) for o in objids]
        offs = np.zeros(len(bs) + 1, np.int64)
        offs[1:] = np.cumsum([len(b) for b in bs])
        blob = b"".join(bs)
        keys = np.empty(len(bs), np.int64)
        _lib.check(_lib.lib().gf_objid_intern(self.handle, blob, offs.ctypes.data, len(bs), keys.ctypes.data),
                   self.ctx.handle, "gf_objid_intern")
        return keys

    def decode_bytes(self, keys):
        """int64 keys -> list of bytes (the Strings' UTF-8)"""
        k = np.ascontiguousarray(np.asarray(keys, np.int64))
        offs = np.zeros(len(k) + 1, np.int64)
        cap = 64 * len(k) + 64
        for _ in range(2):
            buf = C.create_string_buffer(cap)
            st = _lib.lib().gf_objid_decode(self.handle, k.ctypes.data, len(k), buf, cap, offs.ctypes.data)
            if st == _lib.GF_ERR_CAPACITY:
                cap = int(offs[-1])
                continue
            _lib.check(st, self.ctx.handle, "gf_objid_decode")
            raw = buf.raw
            return [raw[offs[i]:offs[i + 1]] for i in range(len(k))]
        raise _lib.GeoFlinkError(_lib.GF_ERR_CAPACITY, "gf_objid_decode")

    def decode(self, keys):
        """int64 keys -> list of str (None for OBJID_NULL: a GeoJSON feature without the objID property)"""
        k = np.asarray(keys, np.int64)
        return [None if kk == _lib.OBJID_NULL else b.decode("utf-8", "surrogateescape")
                for kk, b in zip(k.tolist(), self.decode_bytes(k))]

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and getattr(self, "owned", False) and _lib._lib is not None:
            _lib._lib.gf_objid_dict_destroy(h)
            self.handle = None


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
    objid_dict: Optional[ObjIdDict] = None   # the dictionary of its non-numeric objID keys

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
    def from_points(cls, points, device=None, start=0, end=0, objid_dict: Optional[ObjIdDict] = None):
        """Points with String (or int) objIDs; Strings are mapped to keys by `objid_dict`
        (default: the device context's dictionary)."""
        import torch

        points = list(points)
        dev = torch.cuda.current_device() if device is None else device
        d = objid_dict or ObjIdDict.default(dev)
        x = np.array([p.x for p in points], np.float64)
        y = np.array([p.y for p in points], np.float64)
        # a null objID (Java null: e.g. a GeoJSON feature without the objID property) stays the
        # null key; the String "null" (a JSON null literal's text) is a different objID
        o = np.full(len(points), _lib.OBJID_NULL, np.int64)
        have = [i for i, p in enumerate(points) if p.objID is not None]
        if have:
            o[have] = d.intern([str(points[i].objID) for i in have])
        ts = np.array([p.timeStampMillisec for p in points], np.int64)
        w = cls.from_numpy(x, y, o, ts, device, start, end)
        w.objid_dict = d
        return w

    def objid_strings(self, keys=None):
        """Strings of objID keys (default: every point's)."""
        import torch

        k = self.objID.cpu().numpy() if keys is None else np.asarray(keys, np.int64)
        d = self.objid_dict or ObjIdDict.default(self.x.device.index if self.x.is_cuda else torch.cuda.current_device())
        return d.decode(k)

    def c_struct(self) -> _lib.GfPoints:
        for t in (self.x, self.y):
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("PointWindow tensors must be contiguous CUDA tensors")
        return _lib.GfPoints(self.x.data_ptr(), self.y.data_ptr(), self.objID.data_ptr(),
                             self.timeStampMillisec.data_ptr(), self.n)

    def point(self, i: int, uGrid: Optional[UniformGrid] = None) -> Point:
        i = int(i)
        return Point(self.objid_strings([int(self.objID[i])])[0], float(self.x[i]), float(self.y[i]),
                     int(self.timeStampMillisec[i]), uGrid)
