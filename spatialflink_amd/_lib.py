"""ctypes binding of libgeoflink_hip.so (include/geoflink_hip.h).

The product path: every operator in this package calls the HIP library through this
module.  There is no CPU fallback -- if the library is missing or no GPU is visible the
operators raise instead of silently computing elsewhere.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GF_LIB_PATH") or os.path.join(_HERE, "libgeoflink_hip.so")

GF_OK = 0
OBJID_NUMERIC_MIN, OBJID_NUMERIC_END = -(1 << 62), 1 << 62
OBJID_NULL = (1 << 63) - 1  # GeoJSON feature without the objID property
GF_MERGE_SHARD_MAJOR, GF_MERGE_WINDOW_MAJOR = 0, 1
GF_MERGE_FOREIGN_KEYS = 0x100      # records from other ranks' contexts: dictionary objID keys refused
KNN_STATUS_FOREIGN_KEYS = 2        # merged record status: a window held dictionary keys of another rank
GF_ERR_ARG = -1
GF_ERR_CAPACITY = -2
GF_ERR_HIP = -3
GF_ERR_NOMEM = -4
GF_ERR_LAYERS = -5
GF_ERR_ALIGN = -7
GF_ERR_COMM = -8
GF_COMM_ID_BYTES = 128

METRIC_SQRT = 0
METRIC_HYPOT = 1

FLAG_JOIN_LEGACY = 1
FLAG_JOIN_COARSE = 2
FLAG_GEOJSON_WALK = 4
FLAG_GEOJSON_WAVE = 16
FLAG_GEOJSON_CHECK = 32
FLAG_JOIN_STREAM = 8
(K_KNN_SCAN, K_KNN_SAMPLE, K_KNN_SELECT, K_RANGE_SCAN, K_ASSIGN, K_JOIN_PROBE, K_RANGE_TEST, K_JOIN_BUCKET,
 K_KNN_MERGE, K_CSV_PARSE, K_BUCKET, K_JOIN_COMPACT) = range(12)

# Every symbol include/geoflink_hip.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "gf_abi_version", "gf_build_info", "gf_build_is_product", "gf_status_string", "gf_device_count", "gf_ctx_create", "gf_ctx_destroy",
    "gf_ctx_set_stream", "gf_ctx_stream", "gf_ctx_synchronize", "gf_ctx_join", "gf_ctx_fork", "gf_ctx_last_error", "gf_ctx_set_timing", "gf_ctx_set_timing_period", "gf_ctx_set_flag",
    "gf_geojson_check_counts",
    "gf_ctx_timing", "gf_grid_make", "gf_grid_layers", "gf_cell_of", "gf_format_cell_id", "gf_parse_cell_id",
    "gf_assign_cells", "gf_bucket_by_cell", "gf_range_pp_plan_create", "gf_range_ppoly_plan_create",
    "gf_range_plan_destroy", "gf_range_run", "gf_range_run_batch", "gf_range_plan_stats", "gf_range_plan_set_tuning", "gf_range_plan_set_drain_lanes", "gf_bitmap_to_indices", "gf_bitmap_to_indices_async", "gf_knn_pp_plan_create",
    "gf_knn_ppoly_plan_create",
    "gf_knn_plan_destroy", "gf_knn_plan_set_capacity", "gf_knn_plan_set_index_base", "gf_knn_plan_set_tuning", "gf_knn_plan_set_hint", "gf_knn_plan_set_pipeline", "gf_knn_plan_flush",
    "gf_knn_result_bytes", "gf_knn_enqueue",
    "gf_knn_decode", "gf_knn_run", "gf_knn_merge_dev", "gf_knn_merge_dev_batch", "gf_knn_merge_host",
    "gf_knn_sliding_create", "gf_knn_sliding_destroy", "gf_knn_sliding_geometry", "gf_knn_sliding_push",
    "gf_knn_sliding_flush", "gf_knn_sliding_decode", "gf_range_sliding_create", "gf_range_sliding_destroy",
    "gf_range_sliding_geometry", "gf_range_sliding_push", "gf_pane_bounds", "gf_csv_parse", "gf_csv_parse_dict", "gf_geojson_parse",
    "gf_objid_dict_create", "gf_objid_dict_destroy", "gf_ctx_objid_dict", "gf_objid_dict_size", "gf_objid_intern",
    "gf_objid_decode", "gf_join_pp", "gf_join_pp_async",
    "gf_join_ppoly_plan_create", "gf_join_ppoly_run", "gf_join_ppoly",
    "gf_window_create",
    "gf_window_destroy", "gf_window_upload", "gf_window_points", "gf_synth_uniform", "gf_pinned_alloc",
    "gf_pinned_free", "gf_knn_string_record_bytes", "gf_knn_attach_strings", "gf_knn_merge_dev_strings",
    "gf_knn_string_record_decode", "gf_window_upload_mapped", "gf_shard_by_columns", "gf_gather_points",
    "gf_host_pinned", "gf_comm_available", "gf_comm_unique_id", "gf_comm_create", "gf_comm_create_all",
    "gf_comm_destroy", "gf_comm_info", "gf_comm_last_error", "gf_comm_check", "gf_knn_exchange_batch",
    "gf_knn_exchange_strings_batch", "gf_knn_exchange_group",
]


class GfGrid(C.Structure):
    _fields_ = [("n", C.c_int32), ("reserved", C.c_int32), ("minX", C.c_double), ("maxX", C.c_double),
                ("minY", C.c_double), ("maxY", C.c_double), ("cellLength", C.c_double)]


class GfPoints(C.Structure):
    _fields_ = [("x", C.c_void_p), ("y", C.c_void_p), ("objID", C.c_void_p), ("ts", C.c_void_p),
                ("n", C.c_int64)]


class GfPolygons(C.Structure):
    _fields_ = [("npoly", C.c_int32), ("ring_off", C.c_void_p), ("vert_off", C.c_void_p),
                ("vx", C.c_void_p), ("vy", C.c_void_p)]


class GfKnnHeader(C.Structure):
    _fields_ = [("status", C.c_int32), ("n", C.c_int32), ("k", C.c_int32), ("flags", C.c_int32),
                ("candidates", C.c_int64), ("threshold", C.c_double)]


class GeoFlinkError(RuntimeError):
    def __init__(self, status, msg=""):
        self.status = status
        super().__init__(f"{msg} (status {status}: {status_string(status) if _lib else ''})")


class CandidateLayersError(GeoFlinkError):
    """The reference's System.exit(1): 'candidateNeighboringLayers cannot be 0 or less'
    (UniformGrid.java:272-276), raised instead of terminating the process."""


_lib = None
_lock = threading.Lock()


def lib():
    """Load libgeoflink_hip.so; raise loudly if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()). "
                "There is no CPU fallback for the window-evaluation path.")
        # torch first: it ships its own libamdhip64 (same soname); whichever loads first serves the
        # process, and torch must get the runtime it was built against
        import torch  # noqa: F401

        L = C.CDLL(LIB_PATH)
        P, i32, i64, d, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_double, C.c_size_t
        pi32, pi64, pd = C.POINTER(i32), C.POINTER(i64), C.POINTER(d)
        sig = {
            "gf_abi_version": ([], C.c_int),
            "gf_build_info": ([], C.c_char_p),
            "gf_build_is_product": ([], C.c_int),
            "gf_status_string": ([C.c_int], C.c_char_p),
            "gf_device_count": ([C.POINTER(C.c_int)], C.c_int),
            "gf_ctx_create": ([C.c_int, C.POINTER(P)], C.c_int),
            "gf_ctx_destroy": ([P], None),
            "gf_ctx_set_stream": ([P, P], C.c_int),
            "gf_ctx_stream": ([P], P),
            "gf_ctx_synchronize": ([P], C.c_int),
            "gf_ctx_join": ([P], C.c_int),
            "gf_ctx_fork": ([P], C.c_int),
            "gf_ctx_last_error": ([P], C.c_char_p),
            "gf_ctx_set_timing": ([P, C.c_int], C.c_int),
            "gf_ctx_set_flag": ([P, C.c_int, C.c_int], C.c_int),
            "gf_geojson_check_counts": ([P, P], C.c_int),
            "gf_ctx_set_timing_period": ([P, C.c_int], C.c_int),
            "gf_ctx_timing": ([P, C.c_int, pd, pi64], C.c_int),
            "gf_grid_make": ([i32, d, d, d, d, C.POINTER(GfGrid)], C.c_int),
            "gf_grid_layers": ([C.POINTER(GfGrid), d, pi32, pi32], C.c_int),
            "gf_cell_of": ([C.POINTER(GfGrid), d, d, pi32, pi32], C.c_int),
            "gf_format_cell_id": ([i32, i32, C.c_char_p, i32], C.c_int),
            "gf_parse_cell_id": ([C.c_char_p, pi32, pi32], C.c_int),
            "gf_assign_cells": ([P, C.POINTER(GfGrid), C.POINTER(GfPoints), P, P], C.c_int),
            "gf_bucket_by_cell": ([P, C.POINTER(GfGrid), C.POINTER(GfPoints), P, P], C.c_int),
            "gf_range_pp_plan_create": ([P, C.POINTER(GfGrid), P, P, i32, d, C.c_int, C.c_int, C.POINTER(P)], C.c_int),
            "gf_range_ppoly_plan_create": ([P, C.POINTER(GfGrid), C.POINTER(GfPolygons), d, C.c_int, C.c_int,
                                            C.POINTER(P)], C.c_int),
            "gf_range_plan_destroy": ([P], None),
            "gf_range_run": ([P, C.POINTER(GfPoints), P, P, P], C.c_int),
            "gf_range_run_batch": ([P, i32, C.POINTER(GfPoints), C.POINTER(P), C.POINTER(P), C.POINTER(P), pi64,
                                    C.POINTER(P)], C.c_int),
            "gf_range_plan_stats": ([P, pi64, pi64, pi64, pi64], C.c_int),
            "gf_range_plan_set_tuning": ([P, C.c_int32, C.c_int32], C.c_int),
            "gf_range_plan_set_drain_lanes": ([P, i32], C.c_int),
            "gf_bitmap_to_indices": ([P, P, i64, P, i64, pi64], C.c_int),
            "gf_bitmap_to_indices_async": ([P, P, i64, P, i64, P], C.c_int),
            "gf_knn_pp_plan_create": ([P, C.POINTER(GfGrid), d, d, d, i32, C.c_int, C.POINTER(P)], C.c_int),
            "gf_knn_ppoly_plan_create": ([P, C.POINTER(GfGrid), C.POINTER(GfPolygons), d, i32, C.c_int, C.c_int,
                                          C.POINTER(P)], C.c_int),
            "gf_knn_plan_destroy": ([P], None),
            "gf_knn_plan_set_capacity": ([P, i64], C.c_int),
            "gf_knn_plan_set_index_base": ([P, i64], C.c_int),
            "gf_knn_plan_set_tuning": ([P, i32, i32, i32], C.c_int),
            "gf_knn_plan_set_hint": ([P, C.c_int], C.c_int),
            "gf_knn_plan_set_pipeline": ([P, C.c_int], C.c_int),
            "gf_knn_plan_flush": ([P], C.c_int),
            "gf_knn_result_bytes": ([i32], sz),
            "gf_knn_enqueue": ([P, C.POINTER(GfPoints), P], C.c_int),
            "gf_knn_decode": ([P, C.POINTER(GfPoints), P, P, P, P, pi32], C.c_int),
            "gf_knn_run": ([P, C.POINTER(GfPoints), P, P, P, pi32], C.c_int),
            "gf_knn_merge_dev": ([P, i32, P, i32, P], C.c_int),
            "gf_knn_merge_dev_batch": ([P, i32, P, i32, i32, i32, P], C.c_int),
            "gf_knn_merge_host": ([i32, i32, P, P, P, P, P, P, P, pi32], C.c_int),
            "gf_knn_sliding_create": ([P, i64, i64, C.POINTER(P)], C.c_int),
            "gf_knn_sliding_destroy": ([P], None),
            "gf_knn_sliding_geometry": ([P, pi64, pi32, pi32, pi32], C.c_int),
            "gf_knn_sliding_push": ([P, i64, C.POINTER(GfPoints), P, pi32, pi64], C.c_int),
            "gf_knn_sliding_flush": ([P], C.c_int),
            "gf_knn_sliding_decode": ([P, i64, P, P, P, P, pi32], C.c_int),
            "gf_range_sliding_create": ([P, i64, i64, C.POINTER(P)], C.c_int),
            "gf_range_sliding_destroy": ([P], None),
            "gf_range_sliding_geometry": ([P, pi64, pi32, pi32], C.c_int),
            "gf_range_sliding_push": ([P, i64, C.POINTER(GfPoints), P, i64, P, pi32, pi64, pi64], C.c_int),
            "gf_pane_bounds": ([P, P, i64, i64, i64, i32, P], C.c_int),
            "gf_csv_parse": ([P, P, i64, P, C.POINTER(GfGrid), P, P, P, P, P, P, i64, pi64, pi64, pi32], C.c_int),
            "gf_geojson_parse": ([P, P, P, i64, P, C.POINTER(GfGrid), P, P, P, P, P, P, i64, pi64, pi64, pi32],
                                 C.c_int),
            "gf_csv_parse_dict": ([P, P, P, i64, P, C.POINTER(GfGrid), P, P, P, P, P, P, i64, pi64, pi64, pi32],
                                  C.c_int),
            "gf_objid_dict_create": ([P, C.POINTER(P)], C.c_int),
            "gf_objid_dict_destroy": ([P], None),
            "gf_ctx_objid_dict": ([P, C.POINTER(P)], C.c_int),
            "gf_objid_dict_size": ([P, pi64], C.c_int),
            "gf_objid_intern": ([P, C.c_char_p, P, i64, P], C.c_int),
            "gf_objid_decode": ([P, P, i64, P, i64, P], C.c_int),
            "gf_join_pp": ([P, C.POINTER(GfGrid), C.POINTER(GfGrid), C.POINTER(GfPoints), C.POINTER(GfPoints), d,
                            C.c_int, C.c_int, P, i64, pi64], C.c_int),
            "gf_join_pp_async": ([P, C.POINTER(GfGrid), C.POINTER(GfGrid), C.POINTER(GfPoints), C.POINTER(GfPoints), d,
                                  C.c_int, C.c_int, P, i64, P], C.c_int),
            "gf_join_ppoly_plan_create": ([P, C.POINTER(GfGrid), C.POINTER(GfPolygons), d, C.c_int, C.c_int,
                                           C.POINTER(P)], C.c_int),
            "gf_join_ppoly_run": ([P, C.POINTER(GfGrid), C.POINTER(GfPoints), P, i64, pi64], C.c_int),
            "gf_join_ppoly": ([P, C.POINTER(GfGrid), C.POINTER(GfGrid), C.POINTER(GfPoints), C.POINTER(GfPolygons), d,
                               C.c_int, C.c_int, P, i64, pi64], C.c_int),
            "gf_window_create": ([P, i64, C.POINTER(P)], C.c_int),
            "gf_window_destroy": ([P], None),
            "gf_window_upload": ([P, P, P, P, P, i64], C.c_int),
            "gf_window_points": ([P, C.POINTER(GfPoints)], C.c_int),
            "gf_window_upload_mapped": ([P, P, P, P, i64], C.c_int),
            "gf_shard_by_columns": ([P, C.POINTER(GfGrid), C.POINTER(GfPoints), i32, P, P, P], C.c_int),
            "gf_gather_points": ([P, C.POINTER(GfPoints), P, i64, i64, P, P, P, P], C.c_int),
            "gf_host_pinned": ([P, C.POINTER(C.c_int)], C.c_int),
            "gf_synth_uniform": ([i64, i64, d, d, d, d, P, P], C.c_int),
            "gf_pinned_alloc": ([sz, C.POINTER(P)], C.c_int),
            "gf_pinned_free": ([P], None),
            "gf_knn_string_record_bytes": ([i32, i64], sz),
            "gf_knn_attach_strings": ([P, i32, P, i32, i64, P], C.c_int),
            "gf_knn_merge_dev_strings": ([P, i32, i64, P, i32, i32, i32, P], C.c_int),
            "gf_knn_string_record_decode": ([P, i32, i64, pi32, P, P, P, P, i64, P, pi32], C.c_int),
            "gf_comm_available": ([], C.c_int),
            "gf_comm_unique_id": ([P], C.c_int),
            "gf_comm_create": ([P, i32, i32, C.c_int, C.POINTER(P)], C.c_int),
            "gf_comm_create_all": ([i32, P, P], C.c_int),
            "gf_comm_destroy": ([P], None),
            "gf_comm_info": ([P, pi32, pi32, C.POINTER(C.c_int)], C.c_int),
            "gf_comm_last_error": ([P], C.c_char_p),
            "gf_comm_check": ([P], C.c_int),
            "gf_knn_exchange_batch": ([P, P, i32, P, i32, P], C.c_int),
            "gf_knn_exchange_strings_batch": ([P, P, i32, i64, P, i32, P], C.c_int),
            "gf_knn_exchange_group": ([i32, P, P, i32, P, i32, P], C.c_int),
        }
        for name, (argt, rest) in sig.items():
            if os.environ.get("GF_LIB_PATH") and not hasattr(L, name):
                continue  # an older build under A/B (tools/gpu_ab.sh): entries added since are absent
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = rest
        _lib = L
        return _lib


def status_string(s):
    return lib().gf_status_string(int(s)).decode()


def check(status, ctx=None, what=""):
    if status == GF_OK:
        return
    detail = ""
    if ctx is not None:
        try:
            detail = lib().gf_ctx_last_error(ctx).decode()
        except Exception:  # noqa: BLE001
            detail = ""
    msg = f"{what}: {detail}" if detail else what
    if status == GF_ERR_LAYERS:
        raise CandidateLayersError(status, msg or "candidateNeighboringLayers cannot be 0 or less")
    if status == GF_ERR_ARG:
        raise ValueError(f"{msg} (IllegalArgumentException)")
    raise GeoFlinkError(status, msg)


class Context:
    """One gf_ctx per (device, thread) -- the reference's per-subtask operator instance."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        st = lib().gf_ctx_create(int(device), C.byref(h))
        if st != GF_OK:
            raise GeoFlinkError(st, f"gf_ctx_create(device={device}) failed: is a GPU visible?")
        self.handle = h
        self.device = device

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib is not None:
            _lib.gf_ctx_destroy(h)
            self.handle = None

    def set_stream(self, stream_ptr: int | None):
        check(lib().gf_ctx_set_stream(self.handle, C.c_void_p(stream_ptr or 0)), self.handle, "set_stream")

    def synchronize(self):
        check(lib().gf_ctx_synchronize(self.handle), self.handle, "synchronize")

    def set_timing(self, mask: int):
        """mask: bitmask of (1 << K_*) kernels whose launches are bracketed by HIP events."""
        check(lib().gf_ctx_set_timing(self.handle, int(mask)), self.handle, "set_timing")

    def set_timing_period(self, period: int):
        check(lib().gf_ctx_set_timing_period(self.handle, int(period)), self.handle, "set_timing_period")

    def timing(self, kernel_id: int):
        ms, n = C.c_double(), C.c_int64()
        check(lib().gf_ctx_timing(self.handle, int(kernel_id), C.byref(ms), C.byref(n)), self.handle, "timing")
        return ms.value, n.value


_ctx_cache: dict = {}


def context(device: int | None = None) -> Context:
    """The calling thread's context for `device` (default: torch's current device), bound to
    torch's current stream so library work orders naturally with torch work."""
    import torch

    if device is None:
        device = torch.cuda.current_device()
    key = (int(device), threading.get_ident())
    ctx = _ctx_cache.get(key)
    if ctx is None:
        ctx = Context(int(device))
        _ctx_cache[key] = ctx
    ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)
    return ctx


def device_count() -> int:
    n = C.c_int()
    lib().gf_device_count(C.byref(n))
    return n.value
