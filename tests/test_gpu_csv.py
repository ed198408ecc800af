"""GPU parity of the CSV/TSV ingest (gf_csv_parse, k_csv.hip) against the oracle's
Deserialization.CSVTSVToTSpatial restatement: bit-identical x, y, ts; the objID Strings
(Deserialization.java:317) recovered exactly from the keys, equal keys <=> equal Strings; cells
equal to the oracle's assignGridCellID; the same first bad line and kind on malformed input."""
import numpy as np
import pytest

from conftest import BEIJING
from csv_gen import make_csv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def check_keys(w, o):
    """keys -> the oracle's Strings exactly; equal keys <=> equal Strings; canonical decimals in
    [-2^62, 2^62) are their own key, everything else a dictionary key."""
    keys = w.objID.cpu().numpy()
    assert w.objid_dict.decode_bytes(keys) == o
    first = {}
    for k, s_ in zip(keys.tolist(), o):
        assert first.setdefault(s_, k) == k
    assert len(set(keys.tolist())) == len(first)
    for k, s_ in zip(keys.tolist(), o):
        canon = s_.lstrip(b"-").isdigit() and str(int(s_)).encode() == s_ and -(1 << 62) <= int(s_) < (1 << 62)
        assert (k == int(s_)) if canon else (k < -(1 << 62))


def check(sf, oracle_mod, text, delim, order, grid_n=500, objid_dict=None):
    g = sf.UniformGrid(grid_n, *BEIJING)
    og = oracle_mod.grid(grid_n, *BEIJING)
    parser = sf.Deserialization.CSVTSVToTSpatial(g, None, delim, order)
    w = parser.parse(text, objid_dict=objid_dict)
    x, y, o, t, bl, bk = oracle_mod.csv_parse(text, delim, list(order))
    assert bl == -1
    np.testing.assert_array_equal(w.x.cpu().numpy().view(np.int64), x.view(np.int64))
    np.testing.assert_array_equal(w.y.cpu().numpy().view(np.int64), y.view(np.int64))
    check_keys(w, o)
    np.testing.assert_array_equal(w.timeStampMillisec.cpu().numpy(), t)
    cx, cy = oracle_mod.assign_cells(og, x, y)
    np.testing.assert_array_equal(w.extra["cx"].cpu().numpy(), cx)
    np.testing.assert_array_equal(w.extra["cy"].cpu().numpy(), cy)
    return w


@pytest.mark.parametrize("n,delim,messy,crlf,order,trail,strs", [
    (1_000_000, ",", False, False, (0, 1, 2, 3), True, False),
    (300_000, ",", True, True, (3, 0, 2, 1), False, False),
    (200_000, "\t", True, False, (0, 1, 2, 3), True, True),
    (100_000, ";", True, False, (1, 0, 3, 2), False, True),
    (400_000, ",", True, False, (2, 0, 3, 1), True, True),
])
def test_csv_matches_oracle(sf, oracle_mod, n, delim, messy, crlf, order, trail, strs):
    text, px, py, po, pt = make_csv(n, seed=n % 97, delim=delim, messy=messy, crlf=crlf, order=order,
                                    trailing_newline=trail, string_objids=strs)
    w = check(sf, oracle_mod, text, delim, order, objid_dict=sf.ObjIdDict(0) if strs else None)
    assert w.n == n
    np.testing.assert_array_equal(w.x.cpu().numpy(), px)


def test_csv_objid_strings_across_chunks(sf, oracle_mod):
    """One dictionary over consecutive chunks: a String keeps its key in every chunk; ids are
    given in first-occurrence order (deterministic: the same text gives the same keys)."""
    d1, d2 = sf.ObjIdDict(0), sf.ObjIdDict(0)
    chunks = [make_csv(50_000, seed=s, string_objids=True)[0] for s in range(3)]
    got = {}
    for d in (d1, d2):
        keys = []
        for c in chunks:
            w = check(sf, oracle_mod, c, ",", (0, 1, 2, 3), objid_dict=d)
            keys.append(w.objID.cpu().numpy())
        got[id(d)] = np.concatenate(keys)
        strs = d.decode_bytes(got[id(d)])
        seen = {}
        for k, s_ in zip(got[id(d)].tolist(), strs):
            assert seen.setdefault(s_, k) == k
    np.testing.assert_array_equal(got[id(d1)], got[id(d2)])
    # ids follow first occurrence: dictionary keys appear in increasing order of first sight
    firsts = []
    for k in got[id(d1)].tolist():
        if k < -(1 << 62) and k not in firsts:
            firsts.append(k)
    assert firsts == sorted(firsts) and firsts[0] == -(1 << 63)
    # host intern agrees with the device ingest
    strs = d1.decode_bytes(got[id(d1)][:5000])
    np.testing.assert_array_equal(d1.intern(strs), got[id(d1)][:5000])


def test_csv_short_lines_and_edges(sf, oracle_mod):
    """8-byte lines (more newlines than the first scratch guess), special literals, one line."""
    rng = np.random.default_rng(4)
    vals = ["0", "1.", ".5", "-0.0", "1e-400", "1e400", "NaN", "-Infinity", "4.9e-324", "2.5f", "7D", "+3"]
    lines = [f"{i % 10},{i % 7},{vals[i % len(vals)]},{vals[(i * 5) % len(vals)]}" for i in range(300_000)]
    text = ("\n".join(lines)).encode()
    check(sf, oracle_mod, text, ",", (0, 1, 2, 3))
    check(sf, oracle_mod, b"1,2,116.5,40.25", ",", (0, 1, 2, 3))
    check(sf, oracle_mod, b"5,6,117.0,41.0\n", ",", (0, 1, 2, 3))
    big = ",".join(str(v) for v in rng.integers(0, 9, 500)) + "\n"  # one 1000-byte line, many fields
    check(sf, oracle_mod, (big * 3000).encode(), ",", (3, 7, 400, 11))


@pytest.mark.parametrize("text,line,kind", [
    (b"1,2,3.5,4\n1,2,x,4\n", 1, 1), (b"1,2,3\n", 0, 3), (b"1,2,3,4\n\n5,6,7,8\n", 1, 4), (b"1,2,0x1p3,4\n", 0, 2),
    (b"1,2.5,3,4\n", 0, 1), (b"1,2,3,,\n", 0, 3), (b"9,9,1,1\n" * 70_000 + b"1,2,3,4e\n", 70_000, 1),
    (b"1,x,3\n", 0, 1), (b"1,2,y\n", 0, 1),
])
def test_csv_bad_lines(sf, oracle_mod, text, line, kind):
    *_, bl, bk = oracle_mod.csv_parse(text, ",", [0, 1, 2, 3])
    assert (bl, bk) == (line, kind)
    with pytest.raises(ValueError, match=f"line {line}:"):
        sf.Deserialization.CSVTSVToTSpatial(None, None, ",", (0, 1, 2, 3)).parse(text)


def test_csv_objid_is_a_string(sf, oracle_mod):
    """The reference keeps the objID field as the String (Deserialization.java:317): " 1" (first
    field: the split keeps its leading blank), "007", "+7", "-0", "" and letters are accepted
    and kept apart from "1", "7", "0"."""
    text = b' 1,2,3,4\n1,2,3,4\n007,2,3,4\n7,2,3,4\n+7, 2 ,3,4\n"a"b c ,2,3,4\n,2,3,4\n-0,2,3,4\n0,2,3,4\n'
    w = check(sf, oracle_mod, text, ",", (0, 1, 2, 3), objid_dict=sf.ObjIdDict(0))
    assert w.objid_strings() == [" 1", "1", "007", "7", "+7", "ab c", "", "-0", "0"]


def test_csv_knn_keeps_distinct_string_objids(sf, oracle_mod):
    """CSV -> kNN: the objID dedupe (KNNQuery.java:232-251) is by String, so "007" and "7" (and
    " 7", "+7") are different objects; repeats of one String keep its nearest occurrence."""
    from conftest import QPOINT

    rng = np.random.default_rng(11)
    n = 60_000
    x = QPOINT[0] + rng.uniform(-0.3, 0.3, n)
    y = QPOINT[1] + rng.uniform(-0.3, 0.3, n)
    names = ["7", "007", "+7", "07", "dev-7", " 7"] + [f"obj{i}" for i in range(2000)]
    obj = [names[j] for j in rng.integers(0, len(names), n)]
    # the six look-alikes are the six nearest points
    for i, nm in enumerate(names[:6]):
        x[i], y[i], obj[i] = QPOINT[0] + 1e-5 * (i + 1), QPOINT[1], nm
    text = "".join(f"{o},{i},{float(a)!r},{float(b)!r}\n" for i, (o, a, b) in enumerate(zip(obj, x, y))).encode()
    g = sf.UniformGrid(500, *BEIJING)
    og = oracle_mod.grid(500, *BEIJING)
    d = sf.ObjIdDict(0)
    w = sf.Deserialization.CSVTSVToTSpatial(g, None, ",", (0, 1, 2, 3)).parse(text, objid_dict=d)
    xo, yo, so, to, bl, bk = oracle_mod.csv_parse(text, ",", [0, 1, 2, 3])
    # the oracle dedupes int64 ids: any injective String -> id map gives the same result set
    ids = {s_: i for i, s_ in enumerate(dict.fromkeys(so))}
    oid = np.array([ids[s_] for s_ in so], np.int64)
    q = sf.Point("q", *QPOINT, 0, g)
    res = sf.PointPointKNNQuery(sf.QueryConfiguration(sf.QueryType.WindowBased), g).run(w, q, 0.5, 40)
    st, eo, ed, ei = oracle_mod.knn(og, xo, yo, oid, QPOINT[0], QPOINT[1], 0.5, 40)
    assert st == 0
    np.testing.assert_array_equal(res.dist, ed)
    np.testing.assert_array_equal(np.sort(res.idx), np.sort(ei))
    got = w.objid_strings(res.objID)
    assert got[:6] == ["7", "007", "+7", "07", "dev-7", " 7"]
    assert sorted(got) == sorted(so[i].decode() for i in ei)


def test_csv_capacity_retry(sf, oracle_mod):
    text, *_ = make_csv(5000, seed=2)
    w = sf.Deserialization.CSVTSVToTSpatial(None, None, ",", (0, 1, 2, 3)).parse(text, capacity=10)
    assert w.n == 5000
