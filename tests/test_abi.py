"""CPU: the C-ABI library loads, exports every symbol include/geoflink_hip.h declares, and
its host-side logic (grid, cell IDs, layers, top-k merge, synthetic source) matches the
oracle.  No compute kernels are launched here (no GPU in this container)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import BEIJING, QPOINT, ROOT

import spatialflink_amd as sf
from spatialflink_amd import _lib


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "geoflink_hip.h")).read()
    return sorted(set(re.findall(r"\b(gf_[a-z0-9_]+)\s*\(", txt)))


def test_library_loads():
    L = _lib.lib()
    assert L.gf_abi_version() == 2


def test_exports_match_header():
    declared = header_symbols()
    assert declared == sorted(_lib.EXPORTS)
    L = _lib.lib()
    for s in declared:
        assert hasattr(L, s), s
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\b(gf_[a-z0-9_]+)\b", nm))
    assert set(declared) <= exported


def test_library_is_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"--gfx942" not in blob and b"--gfx90a" not in blob  # gfx950 only, no dual paths


def test_status_strings():
    for s in (0, -1, -2, -3, -4, -5, -7):
        assert _lib.status_string(s)


def test_grid_and_layers(oracle_mod):
    for n in (100, 500, 1000, 37):
        g = sf.UniformGrid(n, *BEIJING)
        og = oracle_mod.grid(n, *BEIJING)
        assert g.getCellLength() == og.cellLength
        for r in (0.0, 0.001, 0.02, 0.05, 0.5, 3.0, -0.1, float("nan"), float("inf")):
            assert (g.getGuaranteedNeighboringLayers(r), g.getCandidateNeighboringLayers(r)) == oracle_mod.layers(og, r)


def test_cell_of_matches_oracle(oracle_mod):
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.uniform(115.0, 118.0, 3000), [np.nan, np.inf, -np.inf, 1e300, -1e300, 115.5, 117.6]])
    ys = np.concatenate([rng.uniform(39.0, 41.5, 3000), [40.0, np.nan, 41.1, 39.6, 1e300, -1e300, 39.6]])
    cx, cy = oracle_mod.assign_cells(og, xs, ys)
    for a, b, c, d in zip(xs, ys, cx, cy):
        assert g.cellOf(a, b) == (int(c), int(d))


def test_cell_id_strings(oracle_mod):
    for (a, b) in [(0, 0), (12, 345), (-1, 5), (99999, 3), (-9999, -1)]:
        s = sf.generateCellIDStr(a, b)
        assert s == oracle_mod.cell_id(a, b)
        assert sf.getIntCellIndices(s) == list(oracle_mod.parse_cell_id(s))
    g = sf.UniformGrid(100, *BEIJING)
    assert g.assignGridCellID(*QPOINT) == oracle_mod.cell_id(*[int(v[0]) for v in oracle_mod.assign_cells(
        oracle_mod.grid(100, *BEIJING), [QPOINT[0]], [QPOINT[1]])])


def test_string_cell_sets_match_oracle(oracle_mod):
    g = sf.UniformGrid(100, *BEIJING)
    og = oracle_mod.grid(100, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    qcx, qcy = g.cellOf(*QPOINT)
    for r in (0.5, 0.05, 0.02):
        G = g.getGuaranteedNeighboringCells(r, q)
        Cc = g.getCandidateNeighboringCells(r, q, G)
        gs, cs = oracle_mod.gc_sets_point(og, r, qcx, qcy)
        assert {tuple(sf.getIntCellIndices(s)) for s in G} == gs
        assert {tuple(sf.getIntCellIndices(s)) for s in Cc} == cs


def test_synthetic_matches_java_random(oracle_mod):
    x, y = sf.synthetic_uniform(42, 5000, *BEIJING)
    ox, oy = oracle_mod.java_random_points(42, 5000, *BEIJING)
    np.testing.assert_array_equal(x, ox)
    np.testing.assert_array_equal(y, oy)


def test_knn_merge_host_is_topk_distinct():
    rng = np.random.default_rng(7)
    lists = []
    for s in range(5):
        m = int(rng.integers(0, 60))
        d = np.sort(rng.choice(np.linspace(0, 1, 40), m))  # ties on purpose
        o = rng.integers(0, 80, m)
        lists.append((o, d, np.arange(m) + 1000 * s))
    for k in (1, 7, 50, 200):
        oo, od, oi = sf.knn_merge_host(k, lists)
        allv = sorted((d, o, i) for (ol, dl, il) in lists for o, d, i in zip(ol, dl, il))
        seen, ref = set(), []
        for d, o, i in allv:
            if o in seen:
                continue
            seen.add(o)
            ref.append((d, o, i))
        ref = ref[:k]
        assert list(zip(od.tolist(), oo.tolist(), oi.tolist())) == [(float(a), int(b), int(c)) for a, b, c in ref]


def test_knn_record_layout():
    for k in (1, 50, 100):
        assert sf.spatialOperators.knn_record_bytes(k) == 32 + 24 * k


def test_polygon_mirror():
    g = sf.UniformGrid(100, *BEIJING)
    p = sf.Polygon([[(116.0, 40.0), (116.05, 40.0), (116.05, 40.04), (116.0, 40.04)]], g)
    assert p.rings[0][0] == p.rings[0][-1]
    assert p.boundingBox == ((116.0, 40.0), (116.05, 40.04))
    a1, b1 = g.cellOf(116.0, 40.0)
    a2, b2 = g.cellOf(116.05, 40.04)
    assert len(p.gridIDsSet) == (a2 - a1 + 1) * (b2 - b1 + 1)
    with pytest.raises(ValueError):
        sf.Polygon([[(0, 0), (1, 0), (0, 1)]], g)


def test_unsupported_query_type_raises():
    conf = sf.QueryConfiguration(sf.QueryType.CountBased)
    q = sf.PointPointRangeQuery(conf, sf.UniformGrid(100, *BEIJING))
    with pytest.raises(ValueError, match="Not yet support"):
        q.run(None, [], 0.5)


def test_gpu_calls_fail_loudly_without_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a device is visible")
    with pytest.raises(Exception):
        _lib.Context(0)


def test_comm_entry_points_without_gpu():
    """The RCCL entry points load lazily (librccl.so.1 dlopen on first use) and refuse bad
    arguments before touching RCCL or a device."""
    import ctypes as C

    from spatialflink_amd import _lib

    L = _lib.lib()
    assert L.gf_comm_available() in (0, 1)
    if not L.gf_comm_available():
        assert L.gf_comm_last_error(None)
    h = C.c_void_p()
    uid = (C.c_uint8 * _lib.GF_COMM_ID_BYTES)()
    assert L.gf_comm_create(uid, 0, 0, 0, C.byref(h)) == _lib.GF_ERR_ARG
    assert L.gf_comm_create(uid, 2, 2, 0, C.byref(h)) == _lib.GF_ERR_ARG
    assert L.gf_comm_create(None, 1, 0, 0, C.byref(h)) == _lib.GF_ERR_ARG
    assert b"bad argument" in L.gf_comm_last_error(None)  # this thread's last failed create
    assert L.gf_comm_unique_id(None) == _lib.GF_ERR_ARG
    assert b"null id" in L.gf_comm_last_error(None)
    hs = (C.c_void_p * 2)()
    assert L.gf_comm_create_all(0, None, hs) == _lib.GF_ERR_ARG
    assert L.gf_knn_exchange_batch(None, None, 50, None, 1, None) == _lib.GF_ERR_ARG
    assert L.gf_knn_exchange_group(0, None, None, 50, None, 1, None) == _lib.GF_ERR_ARG
    assert L.gf_status_string(_lib.GF_ERR_COMM).decode().startswith("RCCL")
