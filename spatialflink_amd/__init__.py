"""spatialflink_amd -- MI355X-native window-evaluation hot path of GeoFlink / SpatialFlink.

The Java operators' per-window bodies (range, kNN, join) run as hand-written HIP kernels
for gfx950 behind the C ABI in include/geoflink_hip.h; this package is the host-side
mirror of the reference operator API (UniformGrid, Point, Polygon, QueryConfiguration,
PointPointRangeQuery, PointPolygonRangeQuery, PointPointKNNQuery, PointPointJoinQuery,
PointPolygonKNNQuery, PointPolygonJoinQuery).
"""
from . import _lib, sharding
from .spatialIndices import UniformGrid, generateCellIDStr, getIntCellIndices, padLeadingZeroesToInt
from .spatialObjects import ObjIdDict, Point, PointWindow, Polygon, PolygonSet
from .spatialOperators import (KNNResult, PinnedRecords, PointPointJoinQuery, PointPointKNNQuery, PointPointRangeQuery,
                               PointPolygonJoinQuery, PointPolygonKNNQuery,
                               PointPolygonRangeQuery, QueryConfiguration, QueryType, RangeResult, assign_cells,
                               bucket_by_cell, knn_merge_host, synthetic_uniform,
                               synthetic_clustered)
from .spatialStreams import Deserialization
from .windows import SlidingKNNQuery, SlidingRangeQuery, SlidingWindows

__all__ = [
    "SlidingWindows", "SlidingKNNQuery", "SlidingRangeQuery", "Deserialization", "PointPolygonKNNQuery", "PointPolygonJoinQuery",
    "UniformGrid", "ObjIdDict", "Point", "Polygon", "PolygonSet", "PointWindow", "QueryType", "QueryConfiguration",
    "PointPointRangeQuery", "PointPolygonRangeQuery", "PointPointKNNQuery", "PointPointJoinQuery", "RangeResult",
    "KNNResult", "PinnedRecords", "knn_merge_host", "assign_cells", "bucket_by_cell", "synthetic_uniform", "synthetic_clustered", "generateCellIDStr",
    "getIntCellIndices", "padLeadingZeroesToInt",
]
