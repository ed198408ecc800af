"""CPU: the oracle's CSV ingest (orc_csv_parse, Deserialization.java:314-322) against an
independent Python restatement of the reference's map: re.split with the same regex
("\\s*" + delimiter + "\\s*", trailing empty strings dropped), the objID field kept as the
String (:317), int() for Long.valueOf, float() for Double.valueOf (both correctly rounded)."""
import re

import numpy as np
import pytest

from csv_gen import make_csv


def py_map(text: bytes, delim, want):
    out = []
    lines = text.decode().split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    for ln in lines:
        if ln.endswith("\r"):
            ln = ln[:-1]
        f = re.split(r"\s*" + re.escape(delim) + r"\s*", ln.replace('"', ""))
        while f and f[-1] == "":
            f.pop()
        out.append((f[want[0]].encode(), int(f[want[1]]), float(f[want[2]].strip().rstrip("fFdD")),
                    float(f[want[3]].strip().rstrip("fFdD"))))
    return out


@pytest.mark.parametrize("delim,messy,crlf,order,strs", [(",", False, False, (0, 1, 2, 3), False),
                                                          (",", True, True, (3, 0, 2, 1), False),
                                                          ("\t", True, False, (0, 1, 2, 3), True),
                                                          (";", True, False, (1, 0, 3, 2), True),
                                                          (",", True, False, (0, 1, 2, 3), True)])
def test_oracle_csv_matches_python_map(oracle_mod, delim, messy, crlf, order, strs):
    text, px, py, po, pt = make_csv(5000, seed=len(delim) + messy, delim=delim, messy=messy, crlf=crlf, order=order,
                                    string_objids=strs)
    want = list(order)
    x, y, o, t, bl, bk = oracle_mod.csv_parse(text, delim, want)
    assert bl == -1
    ref = py_map(text, delim, want)
    assert o == [r[0] for r in ref]
    np.testing.assert_array_equal(t, [r[1] for r in ref])
    np.testing.assert_array_equal(x.view(np.int64), np.array([r[2] for r in ref]).view(np.int64))
    np.testing.assert_array_equal(y.view(np.int64), np.array([r[3] for r in ref]).view(np.int64))
    np.testing.assert_array_equal(x, px)
    if not strs:
        assert o == [str(v).encode() for v in po]


def test_oracle_csv_errors(oracle_mod):
    """Errors in the reference's evaluation order: get(objid), Long.valueOf(get(time)),
    Double.valueOf(get(x)), Double.valueOf(get(y))."""
    cases = [(b"1,2,3.5,4\n1,2,x,4\n", 1, 1), (b"1,2,3\n", 0, 3), (b"1,2,3,4\n\n5,6,7,8\n", 1, 4),
             (b"1,2,0x1p3,4\n", 0, 2), (b"1,2.5,3,4\n", 0, 1), (b"1,2,3,4,,\n", -1, 0),
             (b"1,2,3,,\n", 0, 3),
             (b"1,x,3\n", 0, 1),       # time malformed before the missing y: NumberFormatException
             (b"1,2,y\n", 0, 1),       # x malformed before the missing y
             (b"1,2,3\n", 0, 3)]       # y missing
    for text, line, kind in cases:
        *_, bl, bk = oracle_mod.csv_parse(text, ",", [0, 1, 2, 3])
        assert (bl, bk) == (line, kind), text


def test_oracle_csv_objid_strings(oracle_mod):
    """objID is the String field (Deserialization.java:317), never Long.valueOf: whitespace of
    the first field is kept (the split regex only eats whitespace around delimiters), quotes
    removed, leading zeros / '+' / letters kept as they are."""
    text = b' 1,2,3,4\n007,2,3,4\n+7, 2 ,3,4\n"a"b c ,2,3,4\n,2,3,4\n-0,2,3,4\n'
    x, y, o, t, bl, bk = oracle_mod.csv_parse(text, ",", [0, 1, 2, 3])
    assert (bl, bk) == (-1, 0)
    assert o == [b" 1", b"007", b"+7", b"ab c", b"", b"-0"]
    assert py_map(text, ",", [0, 1, 2, 3])[0][0] == b" 1"
    np.testing.assert_array_equal(t, [2] * 6)
