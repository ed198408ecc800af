"""GPU parity of the CSV/TSV ingest (gf_csv_parse, k_csv.hip) against the oracle's
Deserialization.CSVTSVToTSpatial restatement: bit-identical x, y, objID, ts; cells equal to the
oracle's assignGridCellID; the same first bad line and kind on malformed input."""
import numpy as np
import pytest

from conftest import BEIJING
from csv_gen import make_csv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def check(sf, oracle_mod, text, delim, order, grid_n=500):
    g = sf.UniformGrid(grid_n, *BEIJING)
    og = oracle_mod.grid(grid_n, *BEIJING)
    parser = sf.Deserialization.CSVTSVToTSpatial(g, None, delim, order)
    w = parser.parse(text)
    x, y, o, t, bl, bk = oracle_mod.csv_parse(text, delim, list(order))
    assert bl == -1
    np.testing.assert_array_equal(w.x.cpu().numpy().view(np.int64), x.view(np.int64))
    np.testing.assert_array_equal(w.y.cpu().numpy().view(np.int64), y.view(np.int64))
    np.testing.assert_array_equal(w.objID.cpu().numpy(), o)
    np.testing.assert_array_equal(w.timeStampMillisec.cpu().numpy(), t)
    cx, cy = oracle_mod.assign_cells(og, x, y)
    np.testing.assert_array_equal(w.extra["cx"].cpu().numpy(), cx)
    np.testing.assert_array_equal(w.extra["cy"].cpu().numpy(), cy)
    return w


@pytest.mark.parametrize("n,delim,messy,crlf,order,trail", [
    (1_000_000, ",", False, False, (0, 1, 2, 3), True),
    (300_000, ",", True, True, (3, 0, 2, 1), False),
    (200_000, "\t", True, False, (0, 1, 2, 3), True),
    (100_000, ";", True, False, (1, 0, 3, 2), False),
])
def test_csv_matches_oracle(sf, oracle_mod, n, delim, messy, crlf, order, trail):
    text, px, py, po, pt = make_csv(n, seed=n % 97, delim=delim, messy=messy, crlf=crlf, order=order,
                                    trailing_newline=trail)
    w = check(sf, oracle_mod, text, delim, order)
    assert w.n == n
    np.testing.assert_array_equal(w.x.cpu().numpy(), px)


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
    (b"1,2.5,3,4\n", 0, 1), (b" 1,2,3,4\n", 0, 1), (b"1,2,3,,\n", 0, 3), (b"9,9,1,1\n" * 70_000 + b"1,2,3,4e\n", 70_000, 1),
])
def test_csv_bad_lines(sf, oracle_mod, text, line, kind):
    *_, bl, bk = oracle_mod.csv_parse(text, ",", [0, 1, 2, 3])
    assert (bl, bk) == (line, kind)
    with pytest.raises(ValueError, match=f"line {line}:"):
        sf.Deserialization.CSVTSVToTSpatial(None, None, ",", (0, 1, 2, 3)).parse(text)


def test_csv_capacity_retry(sf, oracle_mod):
    text, *_ = make_csv(5000, seed=2)
    w = sf.Deserialization.CSVTSVToTSpatial(None, None, ",", (0, 1, 2, 3)).parse(text, capacity=10)
    assert w.n == 5000
