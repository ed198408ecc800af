"""The JNI shim's plain-C core (integration/jni/geoflink_shim.c, built as
integration/jni/libgeoflink_shim.so) driven through ctypes exactly as geoflink_jni.c's natives
call it -- one shim_* call per native, host buffers in, host results out -- and checked against
the oracle.  The JNI layer itself needs jni.h (no JDK in the image): the CPU tests below check that
it and GeoFlinkHip.java agree native by native, and that every shim function it calls exists.

Anchors: PointPointKNNQuery.java:132-201 / KNNQuery.java:213-272 (knnWindow), :158,198-200
(sliding), PointPolygonKNNQuery.java:245-317, PointPointRangeQuery.java:150-186,
PointPolygonRangeQuery.java:170-204, JoinQuery.java:73-115, PointPointJoinQuery.java:148-182,
PointPolygonJoinQuery.java:154-213, Deserialization.java:149-211,291-325."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import BEIJING, QPOINT, ROOT

JNI = os.path.join(ROOT, "integration", "jni")
SHIM_SO = os.path.join(JNI, "libgeoflink_shim.so")


def _read(p):
    with open(os.path.join(JNI, p)) as f:
        return f.read()


# ---- CPU: the library and the two JNI sources agree -----------------------------------------
def test_shim_library_exports_header():
    if not os.path.exists(SHIM_SO):
        subprocess.run(["make", "-C", ROOT, "-s", "shim"], check=True)
    declared = set(re.findall(r"\b(shim_\w+)\(", _read("geoflink_shim.h")))
    out = subprocess.run(["nm", "-D", "--defined-only", SHIM_SO], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert declared and declared <= exported, declared - exported


def _java_natives():
    src = _read(os.path.join("GeoFlink", "native_", "GeoFlinkHip.java"))
    out = {}
    for m in re.finditer(r"public static native \S+ (\w+)\(([^)]*)\)", src, re.S):
        params = [p for p in re.sub(r"/\*.*?\*/", "", m.group(2)).split(",") if p.strip()]
        out[m.group(1)] = [p.split()[0] for p in params]
    return out


_JTYPE = {"long": "jlong", "int": "jint", "double": "jdouble", "boolean": "jboolean", "char": "jchar",
          "ByteBuffer": "jobject", "String": "jstring", "long[]": "jlongArray", "int[]": "jintArray",
          "double[]": "jdoubleArray", "byte[]": "jbyteArray"}


def _c_natives():
    src = _read("geoflink_jni.c")
    out = {}
    for m in re.finditer(r"Java_GeoFlink_native_1_GeoFlinkHip_(\w+)\(JNIEnv\* env, jclass cls,?([^)]*)\)", src, re.S):
        out[m.group(1)] = [p.split()[0] for p in m.group(2).split(",") if p.strip()]
    return out


def test_jni_natives_match_java_declarations():
    """Every Java native has a C function with the JNI-mangled name and the parameter types JNI
    maps its Java parameters to, and vice versa."""
    j, c = _java_natives(), _c_natives()
    assert set(j) == set(c), set(j) ^ set(c)
    for name, jp in j.items():
        assert [_JTYPE[t] for t in jp] == c[name], name


def test_jni_calls_only_declared_shim_functions():
    declared = set(re.findall(r"\b(shim_\w+)\(", _read("geoflink_shim.h")))
    called = set(re.findall(r"\b(shim_\w+)\(", _read("geoflink_jni.c")))
    assert called and called <= declared, called - declared
    # the natives the verdict asked for exist: String objIDs, sliding kNN, polygon kNN, GeoJSON schema
    j = _java_natives()
    for n in ("objidIntern", "objidDecode", "knnSlidingPush", "knnSlidingDecode", "knnPolygonPlan"):
        assert n in j, n
    assert j["geoJsonParse"][3:6] == ["String", "String", "String"]


def test_shim_core_has_no_thread_static_state():
    """Device buffers live in the context / plan handles, never in thread- or file-statics
    (two contexts on one thread must not share a window)."""
    for f in ("geoflink_shim.c", "geoflink_jni.c"):
        s = _read(f)
        assert "__thread" not in s and "_Thread_local" not in s, f
        assert not re.search(r"^\s*static\s+(?!int|void|const|jint|jlong|jlongArray|jbyteArray|inline)\w+[\s*]+\w+\s*[=;]", s,
                             re.M), f


# ---- GPU: each shim entry against the oracle -----------------------------------------------
P, i32, i64, d = C.c_void_p, C.c_int32, C.c_int64, C.c_double


@pytest.fixture(scope="module")
def shim(gpu):
    from spatialflink_amd import _lib

    _lib.lib()  # torch's HIP runtime first, then the product library
    assert os.path.exists(SHIM_SO), "build it with `make shim` (part of __graft_entry__.build())"
    S = C.CDLL(SHIM_SO)
    pp = C.POINTER(P)
    S.shim_ctx_create.argtypes = [C.c_int, pp]
    S.shim_ctx_destroy.argtypes = [P]
    S.shim_last_error.argtypes = [P]
    S.shim_last_error.restype = C.c_char_p
    S.shim_objid_intern.argtypes = [P, C.c_char_p, P, i64, P]
    S.shim_objid_decode.argtypes = [P, P, i64, P, i64, P]
    S.shim_knn_plan.argtypes = [P, P, d, d, d, i32, pp]
    S.shim_knn_polygon_plan.argtypes = [P, P, P, d, i32, C.c_int, pp]
    S.shim_knn_destroy.argtypes = [P]
    S.shim_knn_window.argtypes = [P, P, P, P, i64, P, P, P, P]
    S.shim_sliding_create.argtypes = [P, i64, i64, pp]
    S.shim_sliding_destroy.argtypes = [P]
    S.shim_sliding_pane_ms.argtypes = [P, P]
    S.shim_sliding_push.argtypes = [P, i64, P, P, P, i64, P, P]
    S.shim_sliding_flush.argtypes = [P]
    S.shim_sliding_decode.argtypes = [P, i64, P, P, P, P]
    S.shim_range_plan.argtypes = [P, P, P, P, i32, d, C.c_int, pp]
    S.shim_range_polygon_plan.argtypes = [P, P, P, d, C.c_int, pp]
    S.shim_range_destroy.argtypes = [P]
    S.shim_range_window.argtypes = [P, P, P, i64, P, i64, P]
    S.shim_range_sliding_create.argtypes = [P, i64, i64, pp]
    S.shim_range_sliding_destroy.argtypes = [P]
    S.shim_range_sliding_pane_ms.argtypes = [P, P]
    S.shim_range_sliding_push.argtypes = [P, i64, P, P, i64, P, pp, P]
    S.shim_join_window.argtypes = [P, P, P, P, P, i64, P, P, i64, d, C.c_int, pp, P]
    S.shim_polygon_join_window.argtypes = [P, P, P, P, i64, P, d, C.c_int, pp, P]
    S.shim_csv_parse.argtypes = [P, C.c_char_p, i64, P, P, P, P, P, i64, P, P, P]
    S.shim_geojson_parse.argtypes = [P, C.c_char_p, i64, P, P, P, P, P, i64, P, P, P]
    S.shim_pinned_alloc.argtypes = [i64, pp]
    S.shim_pinned_free.argtypes = [P]
    S.shim_comm_unique_id.argtypes = [P]
    S.shim_comm_create.argtypes = [P, P, i32, i32, pp]
    S.shim_comm_create_all.argtypes = [i32, P, P]
    S.shim_comm_destroy.argtypes = [P]
    S.shim_knn_window_sharded.argtypes = [P, P, P, P, P, i64, i64, P, P, P, P]
    return S


@pytest.fixture(scope="module")
def ctx(shim):
    h = P()
    assert shim.shim_ctx_create(0, C.byref(h)) == 0
    yield h
    shim.shim_ctx_destroy(h)


def _a(v):
    return v.ctypes.data_as(P)


def _ok(shim, ctx, st, what):
    assert st == 0, f"{what}: {st} {shim.shim_last_error(ctx)}"


def grid(n, b=BEIJING):
    from spatialflink_amd import _lib

    g = _lib.GfGrid()
    assert _lib.lib().gf_grid_make(n, *b, C.byref(g)) == 0
    return g


def gpolys(OP):
    from spatialflink_amd import _lib

    return _lib.GfPolygons(OP.c.npoly, _a(OP.ring_off), _a(OP.vert_off), _a(OP.vx), _a(OP.vy))


@pytest.mark.gpu
def test_objid_roundtrip(shim, ctx):
    """Point.objID Strings -> keys -> Strings, as a Java caller encodes them (UTF-8 + offsets)."""
    strs = [b"7", b"007", b"-12", b"dev-\xc3\xa9", b"", b"7", b"dev-\xc3\xa9", b"9223372036854775807", b"-0"] * 50
    offs = np.zeros(len(strs) + 1, np.int64)
    offs[1:] = np.cumsum([len(s) for s in strs])
    blob = b"".join(strs)
    keys = np.zeros(len(strs), np.int64)
    _ok(shim, ctx, shim.shim_objid_intern(ctx, blob, _a(offs), len(strs), _a(keys)), "intern")
    assert keys[0] == 7 and keys[2] == -12 and keys[1] < -(1 << 62)
    assert len(set(keys.tolist())) == len(set(strs))
    out_off = np.zeros(len(strs) + 1, np.int64)
    small = C.create_string_buffer(8)
    st = shim.shim_objid_decode(ctx, _a(keys), len(keys), small, 8, _a(out_off))
    assert st == -2 and out_off[-1] == len(blob)  # GF_ERR_CAPACITY, bytes needed
    buf = C.create_string_buffer(int(out_off[-1]) + 1)
    _ok(shim, ctx, shim.shim_objid_decode(ctx, _a(keys), len(keys), buf, len(buf), _a(out_off)), "decode")
    raw = buf.raw
    assert [raw[out_off[i]:out_off[i + 1]] for i in range(len(strs))] == strs


def _knn_window(shim, plan, x, y, o, k):
    oo = np.zeros(k, np.int64); od = np.zeros(k); oi = np.zeros(k, np.int64); m = i32()
    st = shim.shim_knn_window(plan, _a(x), _a(y), _a(o), len(x), _a(oo), _a(od), _a(oi), C.byref(m))
    return st, oo[:m.value], od[:m.value], oi[:m.value]


@pytest.mark.gpu
@pytest.mark.parametrize("k,gn", [(50, 500), (100, 1000)])
def test_knn_window(shim, ctx, oracle_mod, k, gn):
    g, og = grid(gn), oracle_mod.grid(gn, *BEIJING)
    plan = P()
    _ok(shim, ctx, shim.shim_knn_plan(ctx, C.byref(g), QPOINT[0], QPOINT[1], 0.5, k, C.byref(plan)), "plan")
    try:
        for seed, n in ((1, 300_000), (2, 1_100_000), (3, 0), (4, 5)):  # the cached window grows and is reused
            x, y = oracle_mod.java_random_points(seed, n, *BEIJING)
            o = (np.arange(n) % max(1, n // 3)).astype(np.int64)
            st, oo, od, oi = _knn_window(shim, plan, x, y, o, k)
            _ok(shim, ctx, st, "knnWindow")
            est, eo, ed, ei = oracle_mod.knn(og, x, y, o, *QPOINT, 0.5, k)
            assert est == 0
            np.testing.assert_array_equal(oo, eo)
            np.testing.assert_array_equal(od.view(np.int64), ed.view(np.int64))
            np.testing.assert_array_equal(oi, ei)
    finally:
        shim.shim_knn_destroy(plan)


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["rank", "all"])
def test_knn_window_sharded_one_rank(shim, ctx, oracle_mod, form):
    """knnWindowSharded (the multi-GPU drop-in: the windowAll merge as the RCCL record exchange of
    the C ABI) on a one-rank communicator -- ncclCommInitRank from a unique id, or ncclCommInitAll
    -- vs the oracle, with a nonzero index base and a window that overflows the candidate buffer
    (1.1M points stacked on the query point: the record is flagged, every rank re-evaluates
    exactly and the ranks exchange again)."""
    g, og = grid(500), oracle_mod.grid(500, *BEIJING)
    plan, comm = P(), P()
    _ok(shim, ctx, shim.shim_knn_plan(ctx, C.byref(g), QPOINT[0], QPOINT[1], 0.5, 50, C.byref(plan)), "plan")
    if form == "rank":
        uid = (C.c_uint8 * 128)()
        assert shim.shim_comm_unique_id(uid) == 0
        _ok(shim, ctx, shim.shim_comm_create(ctx, uid, 1, 0, C.byref(comm)), "commCreate")
    else:
        devs, hs = (C.c_int * 1)(0), (P * 1)()
        assert shim.shim_comm_create_all(1, devs, hs) == 0
        comm = P(hs[0])
    try:
        rng = np.random.default_rng(9)
        for seed, n, base, stacked in ((11, 400_000, 0, 0), (12, 300_000, 1_000, 0), (13, 100_000, 7, 1_100_000)):
            x, y = oracle_mod.java_random_points(seed, n, *BEIJING)
            if stacked:
                x = np.concatenate([x, np.full(stacked, QPOINT[0])])
                y = np.concatenate([y, np.full(stacked, QPOINT[1])])
            o = (rng.permutation(len(x)) % max(1, len(x) * 2 // 3)).astype(np.int64)
            oo = np.zeros(50, np.int64); od = np.zeros(50); oi = np.zeros(50, np.int64); m = i32()
            st = shim.shim_knn_window_sharded(plan, comm, _a(x), _a(y), _a(o), len(x), base, _a(oo), _a(od), _a(oi),
                                              C.byref(m))
            _ok(shim, ctx, st, "knnWindowSharded")
            est, eo, ed, ei = oracle_mod.knn(og, x, y, o, *QPOINT, 0.5, 50)
            assert est == 0
            np.testing.assert_array_equal(oo[:m.value], eo)
            np.testing.assert_array_equal(od[:m.value].view(np.int64), ed.view(np.int64))
            np.testing.assert_array_equal(oi[:m.value], ei + base)
    finally:
        shim.shim_comm_destroy(comm)
        shim.shim_knn_destroy(plan)


@pytest.mark.gpu
def test_knn_window_pinned_objid(shim, ctx, oracle_mod):
    """knnWindow with the objID column in pinned memory (pinnedBuffer on the Java side): the shim
    detects it (gf_host_pinned) and uploads x, y only (gf_window_upload_mapped) -- the kernels read
    the candidates' keys in place.  Same records as the copied path; windows grow and shrink."""
    g, og = grid(500), oracle_mod.grid(500, *BEIJING)
    plan = P()
    _ok(shim, ctx, shim.shim_knn_plan(ctx, C.byref(g), QPOINT[0], QPOINT[1], 0.5, 50, C.byref(plan)), "plan")
    cap = 1_300_000
    buf = P()
    _ok(shim, ctx, shim.shim_pinned_alloc(8 * cap, C.byref(buf)), "pinned")
    pinned = np.ctypeslib.as_array((C.c_int64 * cap).from_address(buf.value))
    try:
        for seed, n in ((5, 1_200_000), (6, 300_000), (7, 1_300_000)):
            x, y = oracle_mod.java_random_points(seed, n, *BEIJING)
            o = (np.random.default_rng(seed).permutation(n) % (n // 2)).astype(np.int64)
            pinned[:n] = o
            oo = np.zeros(50, np.int64); od = np.zeros(50); oi = np.zeros(50, np.int64); m = i32()
            st = shim.shim_knn_window(plan, _a(x), _a(y), buf, n, _a(oo), _a(od), _a(oi), C.byref(m))
            _ok(shim, ctx, st, "knnWindow pinned")
            est, eo, ed, ei = oracle_mod.knn(og, x, y, o, *QPOINT, 0.5, 50)
            np.testing.assert_array_equal(oo[:m.value], eo)
            np.testing.assert_array_equal(od[:m.value].view(np.int64), ed.view(np.int64))
            np.testing.assert_array_equal(oi[:m.value], ei)
    finally:
        shim.shim_knn_destroy(plan)
        shim.shim_pinned_free(buf)


@pytest.mark.gpu
def test_knn_polygon_plan(shim, ctx, oracle_mod):
    g, og = grid(500), oracle_mod.grid(500, *BEIJING)
    ring = [(116.30, 39.85), (116.50, 39.86), (116.52, 40.01), (116.33, 39.99), (116.30, 39.85)]
    OP = oracle_mod.Polygons([[ring]])
    GP = gpolys(OP)
    plan = P()
    _ok(shim, ctx, shim.shim_knn_polygon_plan(ctx, C.byref(g), C.byref(GP), 0.3, 40, 0, C.byref(plan)), "plan")
    try:
        x, y = oracle_mod.java_random_points(5, 800_000, *BEIJING)
        o = np.arange(len(x), dtype=np.int64)
        st, oo, od, oi = _knn_window(shim, plan, x, y, o, 40)
        _ok(shim, ctx, st, "knnWindow(polygon)")
        m, eo, ed, ei = oracle_mod.knn_ppoly(og, x, y, o, OP, 0.3, 40)
        np.testing.assert_array_equal(oo, eo)
        np.testing.assert_array_equal(od.view(np.int64), ed.view(np.int64))
        np.testing.assert_array_equal(oi, ei)
    finally:
        shim.shim_knn_destroy(plan)


@pytest.mark.gpu
def test_sliding_knn(shim, ctx, oracle_mod):
    """C5's shape (k = 100, 1000 x 1000 grid, size 2 x slide): panes pushed as the JNI
    AllWindowFunction's pane trigger would, every fired window decoded and compared with the
    oracle over that window's points."""
    k, size, slide = 100, 2000, 1000
    g, og = grid(1000), oracle_mod.grid(1000, *BEIJING)
    n = 600_000
    x, y = oracle_mod.java_random_points(8, n, *BEIJING)
    rng = np.random.default_rng(8)
    ts = np.sort(rng.integers(0, 9000, n)).astype(np.int64)
    ts[(ts >= 4000) & (ts < 5000)] += 1000  # an empty pane in the middle
    ts.sort()
    o = (rng.permutation(n) % (n // 2)).astype(np.int64)
    plan, s = P(), P()
    _ok(shim, ctx, shim.shim_knn_plan(ctx, C.byref(g), QPOINT[0], QPOINT[1], 0.5, k, C.byref(plan)), "plan")
    try:
        _ok(shim, ctx, shim.shim_sliding_create(plan, size, slide, C.byref(s)), "sliding")
        pane = i64()
        shim.shim_sliding_pane_ms(s, C.byref(pane))
        assert pane.value == 1000
        fired, todo = [], []
        for p in range(int(ts.max()) // 1000 + 1):
            lo, hi = np.searchsorted(ts, [p * 1000, (p + 1) * 1000])
            closed, end = i32(), i64()
            px, py, po = (np.ascontiguousarray(a[lo:hi]) for a in (x, y, o))
            _ok(shim, ctx, shim.shim_sliding_push(s, p, _a(px), _a(py), _a(po), hi - lo, C.byref(closed),
                                                  C.byref(end)), "push")
            for e in todo:  # windows closed by earlier pushes: their records are complete now
                _check_window(shim, ctx, oracle_mod, s, og, e, size, ts, x, y, o, k)
            todo = [end.value] if closed.value else []
            fired += todo
        if p % 2:  # the last window: decoded while pending (decode flushes) or after an explicit flush
            _ok(shim, ctx, shim.shim_sliding_flush(s), "flush")
        for e in todo:
            _check_window(shim, ctx, oracle_mod, s, og, e, size, ts, x, y, o, k)
        assert len(fired) >= 8
    finally:
        if s:
            shim.shim_sliding_destroy(s)
        shim.shim_knn_destroy(plan)


def _check_window(shim, ctx, oracle_mod, s, og, end, size, ts, x, y, o, k):
    oo = np.zeros(k, np.int64); od = np.zeros(k); oi = np.zeros(k, np.int64); m = i32()
    _ok(shim, ctx, shim.shim_sliding_decode(s, end, _a(oo), _a(od), _a(oi), C.byref(m)), "decode")
    lo, hi = np.searchsorted(ts, [end - size, end])
    st, eo, ed, ei = oracle_mod.knn(og, x[lo:hi], y[lo:hi], o[lo:hi], *QPOINT, 0.5, k)
    assert st == 0 and m.value == len(eo)
    np.testing.assert_array_equal(oo[:m.value], eo)
    np.testing.assert_array_equal(od[:m.value].view(np.int64), ed.view(np.int64))
    np.testing.assert_array_equal(oi[:m.value] - lo, ei)  # idx: position in the pushed stream


def _range(shim, plan, x, y, cap):
    out = np.zeros(max(cap, 1), np.int32); cnt = i64()
    st = shim.shim_range_window(plan, _a(x), _a(y), len(x), _a(out), cap, C.byref(cnt))
    return st, out, cnt.value


@pytest.mark.gpu
def test_range_windows(shim, ctx, oracle_mod):
    g, og = grid(100), oracle_mod.grid(100, *BEIJING)
    qx = np.array([QPOINT[0], 116.9, 117.3]); qy = np.array([QPOINT[1], 40.2, 40.9])
    plan = P()
    _ok(shim, ctx, shim.shim_range_plan(ctx, C.byref(g), _a(qx), _a(qy), 3, 0.05, 0, C.byref(plan)), "plan")
    try:
        for seed, n in ((1, 1_000_000), (2, 64), (3, 0)):
            x, y = oracle_mod.java_random_points(seed, n, *BEIJING)
            exp = oracle_mod.range_pp(og, x, y, qx, qy, 0.05)
            st, out, cnt = _range(shim, plan, x, y, n)
            _ok(shim, ctx, st, "rangeWindow")
            assert cnt == len(exp)
            np.testing.assert_array_equal(out[:cnt].astype(np.int64), exp)
        x, y = oracle_mod.java_random_points(1, 1_000_000, *BEIJING)
        st, out, cnt = _range(shim, plan, x, y, 10)  # the JNI rangeWindow's "call again with more"
        assert st == -2 and cnt == len(oracle_mod.range_pp(og, x, y, qx, qy, 0.05))
    finally:
        shim.shim_range_destroy(plan)


@pytest.mark.gpu
def test_range_polygon(shim, ctx, oracle_mod):
    g, og = grid(100), oracle_mod.grid(100, *BEIJING)
    polys = oracle_mod.generate_query_polygons(20, BEIJING[0], BEIJING[2], BEIJING[1], BEIJING[3])
    OP = oracle_mod.Polygons(polys)
    GP = gpolys(OP)
    plan = P()
    _ok(shim, ctx, shim.shim_range_polygon_plan(ctx, C.byref(g), C.byref(GP), 0.01, 0, C.byref(plan)), "plan")
    try:
        x, y = oracle_mod.java_random_points(4, 500_000, *BEIJING)
        exp = oracle_mod.range_ppoly(og, x, y, OP, 0.01)
        st, out, cnt = _range(shim, plan, x, y, len(x))
        _ok(shim, ctx, st, "rangeWindow(polygon)")
        np.testing.assert_array_equal(out[:cnt].astype(np.int64), exp)
    finally:
        shim.shim_range_destroy(plan)


@pytest.mark.gpu
def test_sliding_range(shim, ctx, oracle_mod):
    """rangeSlidingPush's C sequence: panes pushed consecutively (an empty one included), every
    window holding a point compared with the oracle over that window's points."""
    size, slide = 3000, 1000
    g, og = grid(100), oracle_mod.grid(100, *BEIJING)
    qx, qy = np.array([QPOINT[0]]), np.array([QPOINT[1]])
    n = 400_000
    x, y = oracle_mod.java_random_points(12, n, *BEIJING)
    ts = np.sort(np.random.default_rng(12).integers(0, 8000, n)).astype(np.int64)
    keep = (ts < 3000) | (ts >= 4000)
    x, y, ts = x[keep], y[keep], ts[keep]
    plan, s = P(), P()
    _ok(shim, ctx, shim.shim_range_plan(ctx, C.byref(g), _a(qx), _a(qy), 1, 0.05, 0, C.byref(plan)), "plan")
    try:
        _ok(shim, ctx, shim.shim_range_sliding_create(plan, size, slide, C.byref(s)), "create")
        pane = i64()
        shim.shim_range_sliding_pane_ms(s, C.byref(pane))
        assert pane.value == 1000
        fired = 0
        for p in range(int(ts.max()) // 1000 + 3):  # + the empty panes that close the last windows
            lo, hi = np.searchsorted(ts, [p * 1000, (p + 1) * 1000])
            px, py = np.ascontiguousarray(x[lo:hi]), np.ascontiguousarray(y[lo:hi])
            end, idx, cnt = i64(), P(), i64()
            _ok(shim, ctx, shim.shim_range_sliding_push(s, p, _a(px), _a(py), hi - lo, C.byref(end), C.byref(idx),
                                                        C.byref(cnt)), "push")
            if end.value < 0:
                continue
            fired += 1
            wlo, whi = np.searchsorted(ts, [end.value - size, end.value])
            exp = oracle_mod.range_pp(og, x[wlo:whi], y[wlo:whi], qx, qy, 0.05)
            got = (np.ctypeslib.as_array(C.cast(idx, C.POINTER(C.c_uint32)), shape=(cnt.value,)).astype(np.int64)
                   if cnt.value else np.zeros(0, np.int64))
            np.testing.assert_array_equal(got, exp)
        assert fired == 10  # windows ending 1000 .. 10000 all hold a point
    finally:
        if s:
            shim.shim_range_sliding_destroy(s)
        shim.shim_range_destroy(plan)


def _pairs(ptr, m):
    if m == 0:
        return np.zeros((0, 2), np.int64)
    a = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint32)), shape=(2 * m,)).astype(np.int64)
    p = a.reshape(-1, 2)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


def _sorted(p):
    return p[np.lexsort((p[:, 1], p[:, 0]))]


@pytest.mark.gpu
def test_join_windows(shim, ctx, oracle_mod):
    """Two windows of different size on one context (the pairs buffer is sized from the last
    join, then grown and re-run on GF_ERR_CAPACITY)."""
    g, og = grid(100), oracle_mod.grid(100, *BEIJING)
    for seed, no, nq, r in ((1, 200_000, 20_000, 0.01), (2, 1_000_000, 100_000, 0.02), (3, 1000, 0, 0.01)):
        ox, oy = oracle_mod.java_random_points(seed, no, *BEIJING)
        qx, qy = oracle_mod.java_random_points(seed + 100, nq, *BEIJING)
        pairs, m = P(), i64()
        st = shim.shim_join_window(ctx, C.byref(g), C.byref(g), _a(ox), _a(oy), no, _a(qx), _a(qy), nq, r, 0,
                                   C.byref(pairs), C.byref(m))
        _ok(shim, ctx, st, "joinWindow")
        est, exp = oracle_mod.join_pp(og, og, ox, oy, qx, qy, r)
        assert est == 0 and m.value == len(exp)
        np.testing.assert_array_equal(_pairs(pairs, m.value), _sorted(exp))


@pytest.mark.gpu
def test_polygon_join_window(shim, ctx, oracle_mod):
    g, og = grid(100), oracle_mod.grid(100, *BEIJING)
    OP = oracle_mod.Polygons(oracle_mod.generate_query_polygons(30, BEIJING[0], BEIJING[2], BEIJING[1], BEIJING[3]))
    GP = gpolys(OP)
    x, y = oracle_mod.java_random_points(6, 400_000, *BEIJING)
    pairs, m = P(), i64()
    _ok(shim, ctx, shim.shim_polygon_join_window(ctx, C.byref(g), _a(x), _a(y), len(x), C.byref(GP), 0.005, 0,
                                                 C.byref(pairs), C.byref(m)), "polygonJoinWindow")
    exp = oracle_mod.join_ppoly(og, og, x, y, OP, 0.005)
    assert m.value == len(exp)
    np.testing.assert_array_equal(_pairs(pairs, m.value), _sorted(exp))


def _cols(cap):
    return np.zeros(cap), np.zeros(cap), np.zeros(cap, np.int64), np.zeros(cap, np.int64)


def _decode(shim, ctx, keys):
    off = np.zeros(len(keys) + 1, np.int64)
    buf = C.create_string_buffer(64 * len(keys) + 64)
    _ok(shim, ctx, shim.shim_objid_decode(ctx, _a(keys), len(keys), buf, len(buf), _a(off)), "decode")
    return [buf.raw[off[i]:off[i + 1]] for i in range(len(keys))]


@pytest.mark.gpu
def test_csv_parse(shim, ctx, oracle_mod):
    from csv_gen import make_csv
    from spatialflink_amd.spatialStreams import GfCsvSchema

    text, *_ = make_csv(200_000, seed=3, delim=",", messy=True, order=(2, 0, 3, 1), string_objids=True)
    sc = GfCsvSchema(b",", b"\0\0\0", 2, 0, 3, 1)
    x, y, o, t = _cols(200_000)
    n, bl, bk = i64(), i64(), i32()
    _ok(shim, ctx, shim.shim_csv_parse(ctx, text, len(text), C.byref(sc), _a(x), _a(y), _a(o), _a(t), len(x),
                                       C.byref(n), C.byref(bl), C.byref(bk)), "csvParse")
    ex, ey, eo, et, ebl, _ = oracle_mod.csv_parse(text, ",", [2, 0, 3, 1])
    assert ebl == -1 and n.value == len(ex)
    np.testing.assert_array_equal(x.view(np.int64), ex.view(np.int64))
    np.testing.assert_array_equal(y.view(np.int64), ey.view(np.int64))
    np.testing.assert_array_equal(t, et)
    assert _decode(shim, ctx, o) == eo
    # two more lines than the window (the cut line and the inserted one): room for them, so the
    # bad line is reported, not GF_ERR_CAPACITY (the header: capacity is checked first)
    bad = text[:1000] + b"\n1,2,x,4\n" + text[1000:]
    x, y, o, t = _cols(200_008)
    st = shim.shim_csv_parse(ctx, bad, len(bad), C.byref(sc), _a(x), _a(y), _a(o), _a(t), len(x), C.byref(n),
                             C.byref(bl), C.byref(bk))
    *_, ebl, ebk = oracle_mod.csv_parse(bad, ",", [2, 0, 3, 1])
    assert st == -1 and (bl.value, bk.value) == (ebl, ebk)


@pytest.mark.gpu
@pytest.mark.parametrize("date_fmt,tz,vl,props", [(0, 0, 0, (b"oID", b"timestamp")),
                                                 (1, 480, 0, (b"oID", b"timestamp")),
                                                 (1, -300, 1, (b"oID", b"timestamp")),
                                                 (0, 0, 0, (None, None))])
def test_geojson_parse(shim, ctx, oracle_mod, date_fmt, tz, vl, props):
    """propertyObjID, propertyTimeStamp, dateFormat and the zone offset from the caller
    (Deserialization.java:64-70,158-165), not hardcoded."""
    from geojson_gen import lines
    from spatialflink_amd.spatialStreams import GfGeojsonSchema

    text = lines(30 + tz % 7, 20_000, date_fmt, value_lines=bool(vl))
    sc = GfGeojsonSchema(props[0], props[1], date_fmt, tz, vl)
    x, y, o, t = _cols(20_000)
    n, bl, bk = i64(), i64(), i32()
    _ok(shim, ctx, shim.shim_geojson_parse(ctx, text, len(text), C.byref(sc), _a(x), _a(y), _a(o), _a(t), len(x),
                                           C.byref(n), C.byref(bl), C.byref(bk)), "geoJsonParse")
    ex, ey, eo, et, ebl, _ = oracle_mod.geojson_parse(text, *(p.decode() if p else None for p in props), date_fmt, tz,
                                                      value_lines=bool(vl))
    assert ebl == -1 and n.value == len(ex)
    np.testing.assert_array_equal(x.view(np.int64), ex.view(np.int64))
    np.testing.assert_array_equal(y.view(np.int64), ey.view(np.int64))
    np.testing.assert_array_equal(t, et)
    null = np.iinfo(np.int64).max  # GF_OBJID_NULL: the reference's null objID
    assert [None if k == null else s for k, s in zip(o.tolist(), _decode(shim, ctx, o))] == eo


# ---- the Java window functions: their native call order, replayed through the C core ---------
# Per class and method, the GeoFlinkHip natives in source order ("intern" = GeoFlinkHip.intern, the
# Java helper over objidIntern that HipColumns.fill calls for objID columns).  Conditional calls
# are listed as they appear in the source; GPU_SKIPPED names the ones the GPU replay does not take.
JAVA_SEQ = {
    "HipKnnWindowFunction": {"open": ["ctxCreate", "knnPlan"], "grow": ["pinnedFree", "pinnedBuffer"],
                             "apply": ["intern", "knnWindow"],
                             "close": ["pinnedFree", "knnPlanDestroy", "ctxDestroy"]},
    "HipRangeWindowFunction": {"open": ["ctxCreate", "rangePlan", "rangePolygonPlan"],
                               "apply": ["rangeWindow", "rangeWindow", "rangeWindowMulti"],
                               "close": ["rangePlanDestroy", "ctxDestroy"]},
    "HipJoinFunction": {"open": ["ctxCreate"], "coGroup": ["joinWindow"], "close": ["ctxDestroy"]},
    "HipPolygonJoinFunction": {"open": ["ctxCreate"], "coGroup": ["polygonJoinWindow"], "close": ["ctxDestroy"]},
    "HipShardedKnnFunction": {"open": ["ctxCreate", "knnPlan", "commUniqueId", "commCreate", "knnShardedBegin"],
                              "apply": ["intern", "knnShardedEnqueue", "knnShardedResult"],
                              "close": ["commDestroy", "knnPlanDestroy", "ctxDestroy"]},
    "CommRendezvous": {"create": ["commUniqueId", "commCreate"]},
}
# helpers that only read state (not part of a native's action sequence)
_SHIM_QUERIES = {"shim_last_error", "shim_knn_k", "shim_sliding_plan"}


def _java_methods(cls):
    """method name -> its body, for the class's top-level methods (brace matching)"""
    src = re.sub(r"//[^\n]*|/\*.*?\*/", "", _read(os.path.join("GeoFlink", "native_", cls + ".java")), flags=re.S)
    out = {}
    for m in re.finditer(r"\n  (?:public |private |protected |static |final )*[\w<>\[\], ]+ (\w+)\([^)]*\)[^{;]*\{", src):
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        out[m.group(1)] = src[m.end():i]
    return src, out


def _java_native_calls(cls, method):
    src, methods = _java_methods(cls)
    objid_cols = "new HipColumns(true)" in src
    calls = []
    for m in re.finditer(r"GeoFlinkHip\.(\w+)\(|\b\w+\.fill\(|CommRendezvous\.create\(", methods[method]):
        if m.group(1):
            calls.append(m.group(1))
        elif m.group(0).startswith("CommRendezvous"):
            calls.extend(JAVA_SEQ["CommRendezvous"]["create"])
        elif objid_cols:
            calls.append("intern")
    return calls


def _jni_shim_map():
    """native -> the shim_* functions its JNI wrapper calls, in order ("intern" -> objidIntern's)"""
    src = _read("geoflink_jni.c")
    out = {}
    for m in re.finditer(r"Java_GeoFlink_native_1_GeoFlinkHip_(\w+)\(JNIEnv\* env[^{]*\{", src):
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        out[m.group(1)] = [f for f in re.findall(r"\b(shim_\w+)\(", src[m.end():i]) if f not in _SHIM_QUERIES]
    out["intern"] = out["objidIntern"]
    return out


def test_java_functions_call_natives_in_order():
    """Every Java window function's methods call the natives in the order JAVA_SEQ lists (the
    order the GPU replay below drives through the C core), and every native exists with a JNI
    wrapper that calls the shim."""
    jn, jmap = _java_natives(), _jni_shim_map()
    for cls, methods in JAVA_SEQ.items():
        if cls == "CommRendezvous":
            continue
        for method, seq in methods.items():
            assert _java_native_calls(cls, method) == seq, (cls, method, _java_native_calls(cls, method))
            for nat in seq:
                assert nat == "intern" or nat in jn, nat
                assert jmap[nat], f"{nat}: its JNI wrapper calls no shim function"
    assert _java_native_calls("CommRendezvous", "create") == JAVA_SEQ["CommRendezvous"]["create"]
    # the reference's callers are range queries (StreamingJob.java:260,270, MN_Q1.java:63,
    # Q1_HighRisk.java:74): the range function exists for point and polygon query sets
    src, _ = _java_methods("HipRangeWindowFunction")
    assert "Set<Point> queryPoints" in src and "forPolygons(" in src and "Set<Polygon> polygons" in src


class _Recorder:
    """the shim CDLL, recording the shim_* functions called (queries excluded)"""

    def __init__(self, lib):
        self._lib, self.calls = lib, []

    def __getattr__(self, name):
        f = getattr(self._lib, name)
        if name in _SHIM_QUERIES:
            return f

        def rec(*a):
            self.calls.append(name)
            return f(*a)
        return rec


def _expect(cls, method, skip=()):
    jmap = _jni_shim_map()
    seq = [n for n in JAVA_SEQ[cls][method] if n not in skip]
    return [f for n in seq for f in jmap[n]]


def _intern(S, ctx, keys_str):
    offs = np.zeros(len(keys_str) + 1, np.int64)
    offs[1:] = np.cumsum([len(s) for s in keys_str])
    keys = np.zeros(len(keys_str), np.int64)
    _ok(S, ctx, S.shim_objid_intern(ctx, b"".join(keys_str), _a(offs), len(keys_str), _a(keys)), "intern")
    return keys


@pytest.mark.gpu
def test_java_call_sequence_range(shim, oracle_mod):
    """HipRangeWindowFunction, point queries, approximate with |Q| = 3 (the multiplicity list) and
    exact: open / two windows / close replayed in the Java order; the emitted multiset == the
    oracle's (PointPointRangeQuery.java:150-186, the reference's per-query-point emission)."""
    g, og = grid(100), oracle_mod.grid(100, *BEIJING)
    qx = np.array([QPOINT[0], 116.9, 117.3]); qy = np.array([QPOINT[1], 40.2, 40.9])
    for approx in (1, 0):
        S = _Recorder(shim)
        ctx, plan = P(), P()
        assert S.shim_ctx_create(0, C.byref(ctx)) == 0
        _ok(S, ctx, S.shim_range_plan(ctx, C.byref(g), _a(qx), _a(qy), 3, 0.05, approx, C.byref(plan)), "plan")
        assert S.calls == _expect("HipRangeWindowFunction", "open", skip=("rangePolygonPlan",))
        for seed, n in ((21, 600_000), (22, 3000)):
            S.calls.clear()
            x, y = oracle_mod.java_random_points(seed, n, *BEIJING)
            st, out, cnt = _range(S, plan, x, y, max(1, n // 8))  # the first, too-small buffer
            if st == -2:
                st, out, cnt = _range(S, plan, x, y, cnt)
            _ok(S, ctx, st, "rangeWindow")
            multi = np.zeros(max(cnt, 1), np.int32); mc = i64()
            _ok(S, ctx, S.shim_range_window_multi(plan, _a(multi), len(multi), C.byref(mc)), "rangeWindowMulti")
            # rangeWindow, its retry with a large enough buffer only when the first was too small
            exp_calls = _expect("HipRangeWindowFunction", "apply")
            assert S.calls == (exp_calls if cnt > max(1, n // 8) else exp_calls[1:]), S.calls
            emitted = np.repeat(out[:cnt].astype(np.int64),
                                np.where(np.isin(out[:cnt], multi[:mc.value]), 3, 1))
            exp = oracle_mod.range_pp(og, x, y, qx, qy, 0.05, approximate=bool(approx))
            np.testing.assert_array_equal(emitted, np.sort(exp))
            assert (mc.value > 0) == bool(approx)
        S.calls.clear()
        S.shim_range_destroy(plan)
        S.shim_ctx_destroy(ctx)
        assert S.calls == _expect("HipRangeWindowFunction", "close")


@pytest.mark.gpu
def test_java_call_sequence_joins(shim, oracle_mod):
    """HipJoinFunction / HipPolygonJoinFunction: open, one coGroup, close in the Java order; pairs
    == the oracle's (PointPointJoinQuery.java:148-182, PointPolygonJoinQuery.java:154-213)."""
    g, og = grid(100), oracle_mod.grid(100, *BEIJING)
    ox, oy = oracle_mod.java_random_points(31, 300_000, *BEIJING)
    qx, qy = oracle_mod.java_random_points(32, 30_000, *BEIJING)
    OP = oracle_mod.Polygons(oracle_mod.generate_query_polygons(25, BEIJING[0], BEIJING[2], BEIJING[1], BEIJING[3]))
    GP = gpolys(OP)
    for cls in ("HipJoinFunction", "HipPolygonJoinFunction"):
        S = _Recorder(shim)
        ctx = P()
        assert S.shim_ctx_create(0, C.byref(ctx)) == 0
        assert S.calls == _expect(cls, "open")
        S.calls.clear()
        pairs, m = P(), i64()
        if cls == "HipJoinFunction":
            _ok(S, ctx, S.shim_join_window(ctx, C.byref(g), C.byref(g), _a(ox), _a(oy), len(ox), _a(qx), _a(qy),
                                           len(qx), 0.01, 0, C.byref(pairs), C.byref(m)), "joinWindow")
            est, exp = oracle_mod.join_pp(og, og, ox, oy, qx, qy, 0.01)
        else:
            _ok(S, ctx, S.shim_polygon_join_window(ctx, C.byref(g), _a(ox), _a(oy), len(ox), C.byref(GP), 0.005, 0,
                                                   C.byref(pairs), C.byref(m)), "polygonJoinWindow")
            exp = oracle_mod.join_ppoly(og, og, ox, oy, OP, 0.005)
        assert S.calls == _expect(cls, "coGroup")
        np.testing.assert_array_equal(_pairs(pairs, m.value), _sorted(exp))
        S.calls.clear()
        S.shim_ctx_destroy(ctx)
        assert S.calls == _expect(cls, "close")


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3])
def test_java_call_sequence_sharded_knn(shim, oracle_mod, batch):
    """HipShardedKnnFunction on a one-rank communicator (CommRendezvous: unique id + commCreate):
    windows enqueued with String objIDs interned per window, their batch exchanged by String with
    its last window, every window's result read -- == the oracle's kNN of the window (idx global:
    rank << 32 + position; all owned on one rank); a window of 1.1M points stacked on the query
    point overflows the candidate buffer, so its result takes the flagged path (exact
    re-evaluation and a second exchange).  Then the slot-reuse guard and the flush."""
    g, og = grid(500), oracle_mod.grid(500, *BEIJING)
    S = _Recorder(shim)
    S._lib.shim_knn_sharded_begin.argtypes = [P, P, i32, i64]
    S._lib.shim_knn_sharded_enqueue.argtypes = [P, P, P, P, i64, i64, P]
    S._lib.shim_knn_sharded_flush.argtypes = [P]
    S._lib.shim_knn_sharded_result.argtypes = [P, i64, P, P, P, P]
    ctx, plan, comm = P(), P(), P()
    k, base = 50, 0  # rank 0
    assert S.shim_ctx_create(0, C.byref(ctx)) == 0
    _ok(S, ctx, S.shim_knn_plan(ctx, C.byref(g), QPOINT[0], QPOINT[1], 0.5, k, C.byref(plan)), "plan")
    uid = (C.c_uint8 * 128)()
    assert S.shim_comm_unique_id(uid) == 0
    _ok(S, ctx, S.shim_comm_create(ctx, uid, 1, 0, C.byref(comm)), "commCreate")
    _ok(S, ctx, S.shim_knn_sharded_begin(plan, comm, batch, 32 * k + 64), "begin")
    assert S.calls == _expect("HipShardedKnnFunction", "open")  # (rank 0 of CommRendezvous)
    try:
        pending, wins = [], {}
        rng = np.random.default_rng(5)
        specs = [(41, 300_000, 0), (42, 250_000, 1_100_000), (43, 200_000, 0), (44, 5, 0), (45, 350_000, 0), (46, 0, 0)]
        for w, (seed, n, stacked) in enumerate(specs):
            x, y = oracle_mod.java_random_points(seed, n, *BEIJING)
            if stacked:
                x = np.concatenate([x, np.full(stacked, QPOINT[0])]); y = np.concatenate([y, np.full(stacked, QPOINT[1])])
            ids = (rng.permutation(len(x)) % max(1, len(x) * 2 // 3)).astype(np.int64)
            strs = [b"v%d" % i if i % 5 else b"%d" % i for i in ids.tolist()]
            if stacked:  # exact distance ties: broken by dictionary id on a rank (arrival order, as the
                strs = [b"%d" % i for i in ids.tolist()]  # reference's queue), so decimals here (by value)
            S.calls.clear()
            keys = _intern(S, ctx, strs)
            t = i64()
            _ok(S, ctx, S.shim_knn_sharded_enqueue(plan, _a(x), _a(y), _a(keys), len(x), base, C.byref(t)), "enqueue")
            assert t.value == w
            wins[w] = (x, y, ids)
            pending.append(w)
            if (w + 1) % batch:
                assert S.calls == _expect("HipShardedKnnFunction", "apply")[:2]
                continue
            for tw in pending:
                od, oi, ow, m = np.zeros(k), np.zeros(k, np.int64), np.zeros(k, np.int32), i32()
                _ok(S, ctx, S.shim_knn_sharded_result(plan, tw, _a(od), _a(oi), _a(ow), C.byref(m)), "result")
                wx, wy, wid = wins.pop(tw)
                est, eo, ed, ei = oracle_mod.knn(og, wx, wy, wid, *QPOINT, 0.5, k)
                assert est == 0 and m.value == len(eo)
                np.testing.assert_array_equal(od[:m.value].view(np.int64), ed.view(np.int64))
                np.testing.assert_array_equal(wid[oi[:m.value] - base], eo)   # the window's own Points
                assert ow[:m.value].all()
            assert S.calls == _expect("HipShardedKnnFunction", "apply")[:2] + \
                ["shim_knn_sharded_result"] * len(pending)
            pending.clear()
        if batch > 1:  # an unread window blocks its slot 2B tickets later; a flush exchanges a partial batch
            x, y = oracle_mod.java_random_points(50, 1000, *BEIJING)
            keys = np.arange(1000, dtype=np.int64)
            t = i64()
            for _ in range(2 * batch):
                _ok(S, ctx, S.shim_knn_sharded_enqueue(plan, _a(x), _a(y), _a(keys), 1000, base, C.byref(t)), "fill")
            first = t.value - 2 * batch + 1
            assert S.shim_knn_sharded_enqueue(plan, _a(x), _a(y), _a(keys), 1000, base, C.byref(t)) == -1
            od, oi, ow, m = np.zeros(k), np.zeros(k, np.int64), np.zeros(k, np.int32), i32()
            for tw in range(first, first + 2 * batch):
                _ok(S, ctx, S.shim_knn_sharded_result(plan, tw, _a(od), _a(oi), _a(ow), C.byref(m)), "drain")
            _ok(S, ctx, S.shim_knn_sharded_enqueue(plan, _a(x), _a(y), _a(keys), 1000, base, C.byref(t)), "partial")
            assert S.shim_knn_sharded_result(plan, t.value, _a(od), _a(oi), _a(ow), C.byref(m)) == -1  # not exchanged
            _ok(S, ctx, S.shim_knn_sharded_flush(plan), "flush")
            _ok(S, ctx, S.shim_knn_sharded_result(plan, t.value, _a(od), _a(oi), _a(ow), C.byref(m)), "after flush")
            est, eo, ed, ei = oracle_mod.knn(og, x, y, keys, *QPOINT, 0.5, k)
            np.testing.assert_array_equal(od[:m.value].view(np.int64), ed.view(np.int64))
    finally:
        S.calls.clear()
        S.shim_comm_destroy(comm)
        S.shim_knn_destroy(plan)
        S.shim_ctx_destroy(ctx)
        assert S.calls == _expect("HipShardedKnnFunction", "close")
