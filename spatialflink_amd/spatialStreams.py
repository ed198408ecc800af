"""Ingest -- mirror of GeoFlink.spatialStreams.Deserialization for the CSV/TSV point stream
(Deserialization.CSVTSVToTSpatial, Deserialization.java:291-325) and the GeoJSON point stream
(Deserialization.GeoJSONToTSpatial, Deserialization.java:149-211), run on the GPU.

The reference maps each text line to a Point with String.split + Long.valueOf +
Double.valueOf and assigns its grid cell in the Point constructor (Point.java:98).  Here a whole
chunk of lines (device bytes, or host bytes uploaded once) becomes the window's SoA in one call:
gf_csv_parse (k_csv.hip) finds the lines, splits the fields with the reference's
"\\s*delim\\s*" rule, parses the numbers correctly rounded on the device and writes x, y,
objID keys (the objID field is a String, :317 -- canonical decimals are their value, any other
String goes through the device dictionary, k_objid.hip), ts and the cells (cx, cy) -- no
per-point host work.  A bad line raises ValueError naming
it (the reference's map throws NumberFormatException / IndexOutOfBoundsException).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .spatialObjects import ObjIdDict, PointWindow


class GfCsvSchema(C.Structure):
    _fields_ = [("delimiter", C.c_char), ("reserved", C.c_char * 3), ("objid_field", C.c_int32),
                ("time_field", C.c_int32), ("x_field", C.c_int32), ("y_field", C.c_int32)]


CSV_KINDS = {0: "ok", 1: "NumberFormatException", 2: "unsupported numeric literal", 3: "missing field",
             4: "empty line"}


def device_text(text, device=None):
    """bytes / bytearray / numpy uint8 -> a 16-byte-aligned device uint8 tensor (torch allocations
    are 256-B aligned); a device uint8 tensor is returned as is."""
    import torch

    if isinstance(text, torch.Tensor):
        return text
    # bytearray: a writable buffer (torch.from_numpy of a read-only array is undefined behaviour)
    arr = np.frombuffer(bytearray(text), np.uint8) if not isinstance(text, np.ndarray) else text
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    return torch.from_numpy(np.ascontiguousarray(arr)).to(dev)


class GfGeojsonSchema(C.Structure):
    _fields_ = [("objid_property", C.c_char_p), ("time_property", C.c_char_p), ("date_format", C.c_int32),
                ("tz_offset_minutes", C.c_int32), ("value_lines", C.c_int32)]


GEOJSON_DATE_FORMATS = {None: 0, "yyyy-MM-dd HH:mm:ss": 1}


def _parse_lines(fn, schema, uGrid, text, device, capacity, objid_dict):
    import torch

    t = device_text(text, device)
    dev = t.device
    ctx = _lib.context(dev.index)
    d = objid_dict or ObjIdDict.default(dev.index)
    n = int(t.numel())
    cap = capacity if capacity is not None else max(1, n // 8 + 1)
    nout, bl, bk = C.c_int64(), C.c_int64(), C.c_int32()
    while True:
        x = torch.empty(cap, dtype=torch.float64, device=dev)
        y = torch.empty(cap, dtype=torch.float64, device=dev)
        o = torch.empty(cap, dtype=torch.int64, device=dev)
        ts = torch.empty(cap, dtype=torch.int64, device=dev)
        cx = torch.empty(cap, dtype=torch.int32, device=dev) if uGrid is not None else None
        cy = torch.empty(cap, dtype=torch.int32, device=dev) if uGrid is not None else None
        st = fn(ctx.handle, d.handle, C.c_void_p(t.data_ptr()), n, C.byref(schema),
                C.byref(uGrid.c_grid) if uGrid is not None else None, x.data_ptr(), y.data_ptr(), o.data_ptr(),
                ts.data_ptr(), cx.data_ptr() if cx is not None else None, cy.data_ptr() if cy is not None else None,
                cap, C.byref(nout), C.byref(bl), C.byref(bk))
        if st == _lib.GF_ERR_CAPACITY:
            cap = nout.value
            continue
        if st == _lib.GF_ERR_ARG and bl.value >= 0:
            raise ValueError(f"line {bl.value}: {CSV_KINDS.get(bk.value, bk.value)}")
        _lib.check(st, ctx.handle, "parse")
        break
    m = nout.value
    w = PointWindow(x[:m], y[:m], o[:m], ts[:m], objid_dict=d)
    if cx is not None:
        w.extra["cx"], w.extra["cy"] = cx[:m], cy[:m]
    return w


class Deserialization:
    class GeoJSONToTSpatial:
        """GeoJSONToTSpatial(uGrid, dateFormat, propertyTimeStamp, propertyObjID)
        (Deserialization.java:149-211) over lines of GeoJSON, run on the GPU (gf_geojson_parse):
        one Kafka key/value record ({"key": .., "value": ..}, the ObjectNode the map receives) per
        line, or with value_lines=True the record's value itself (a Feature as the reference's
        Serialization writes it).  dateFormat: None (the time property is integer milliseconds)
        or "yyyy-MM-dd HH:mm:ss" in a fixed UTC offset `tz_offset_minutes` (the reference JVM's
        default zone).  A feature without the objID property has objID None (key OBJID_NULL)."""

        def __init__(self, uGrid=None, dateFormat=None, propertyTimeStamp=None, propertyObjID=None,
                     tz_offset_minutes=0, value_lines=False):
            if dateFormat not in GEOJSON_DATE_FORMATS:
                raise ValueError(f"dateFormat {dateFormat!r}: supported {list(GEOJSON_DATE_FORMATS)}")
            self.uGrid = uGrid
            self._names = (propertyObjID.encode() if propertyObjID else None,
                           propertyTimeStamp.encode() if propertyTimeStamp else None)
            self.schema = GfGeojsonSchema(self._names[0], self._names[1], GEOJSON_DATE_FORMATS[dateFormat],
                                          int(tz_offset_minutes), int(bool(value_lines)))

        def parse(self, text, device=None, capacity=None, objid_dict: ObjIdDict = None) -> PointWindow:
            return _parse_lines(_lib.lib().gf_geojson_parse, self.schema, self.uGrid, text, device, capacity,
                                objid_dict)

    class CSVTSVToTSpatial:
        """CSVTSVToTSpatial(uGrid, dateFormat, delimiter, csvTsvSchemaAttr) -- csvTsvSchemaAttr
        lists the field indices of objID, timestamp, x, y (Deserialization.java:314-322).
        dateFormat is unused by the reference's map (the time field is Long.valueOf)."""

        def __init__(self, uGrid=None, dateFormat=None, delimiter=",", csvTsvSchemaAttr=(0, 1, 2, 3)):
            if len(delimiter) != 1:
                raise ValueError("single-character delimiters only")
            self.uGrid = uGrid
            self.delimiter = delimiter
            a = list(csvTsvSchemaAttr)
            self.schema = GfCsvSchema(delimiter.encode(), b"\0\0\0", a[0], a[1], a[2], a[3])

        def parse(self, text, device=None, capacity=None, objid_dict: ObjIdDict = None) -> PointWindow:
            """All lines of `text` -> one PointWindow (extra: cx, cy when a grid is set).  objID
            Strings become keys of `objid_dict` (default: the device context's dictionary)."""
            return _parse_lines(_lib.lib().gf_csv_parse_dict, self.schema, self.uGrid, text, device, capacity,
                                objid_dict)
