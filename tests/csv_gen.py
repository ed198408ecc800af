"""Synthetic CSV/TSV text for the ingest tests and the C1 ingest bench: one point per line,
objID, timestamp, x, y in the ATC-style schema of Deserialization.java:311-312 (fields may be
reordered by csvTsvSchemaAttr), with the variations the reference's map tolerates."""
import numpy as np


def fmt_double(v, style):
    if style == 0:
        return repr(float(v))            # shortest round trip (Java Double.toString digits)
    if style == 1:
        return f"{v:.6f}"                # fixed, like GPS dumps
    if style == 2:
        return f"{v:.17e}"               # 18 significant digits, exponent
    if style == 3:
        return f"{v:.3f}"
    return f"{v:.15g}"


def objid_pool(rng, m):
    """m distinct objID Strings of the kinds the reference keeps apart (String objIDs,
    Deserialization.java:317): canonical decimals, leading zeros, '+', "-0", values past the
    numeric key range, device names, UTF-8, embedded spaces."""
    kinds = [lambda i: str(int(rng.integers(-10**15, 10**15))),
             lambda i: "0" * int(rng.integers(1, 4)) + str(int(rng.integers(0, 10**6))),
             lambda i: "+" + str(int(rng.integers(0, 10**6))),
             lambda i: f"dev-{i}",
             lambda i: f"SNCB_{int(rng.integers(0, 2**40)):x}",
             lambda i: str(int(rng.integers(2**62, 2**63 - 1))),
             lambda i: "-" + str(int(rng.integers(2**62 + 1, 2**63))),
             lambda i: f"trein {i} \u00e9",
             lambda i: str(i % 1000)]
    out = []
    seen = set()
    i = 0
    while len(out) < m:
        v = kinds[i % len(kinds)](i)
        i += 1
        if v not in seen:
            seen.add(v)
            out.append(v)
    return out + ["0", "-0", "7", "007", "+7"]


def make_csv(n, seed=0, delim=",", messy=False, order=(0, 1, 2, 3), crlf=False, trailing_newline=True,
             string_objids=False):
    """-> (bytes, x, y, objID, ts): the exact values are those a correct parser must return
    (objID: int64 values, or with string_objids the objID field texts -- repeated Strings; the
    Strings the reference keeps come from the oracle / the Python map)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(115.5, 117.6, n)
    y = rng.uniform(39.6, 41.1, n)
    obj = rng.integers(-10**12, 10**12, n)
    ts = rng.integers(0, 2 * 10**12, n)
    if string_objids:
        pool = objid_pool(rng, max(8, n // 4))
        obj_txt = [pool[j] for j in rng.integers(0, len(pool), n)]
    styles = rng.integers(0, 5, n) if messy else np.zeros(n, np.int64)
    lines = []
    for i in range(n):
        o = obj_txt[i] if string_objids else str(int(obj[i]))
        f = [o, str(int(ts[i])), fmt_double(x[i], styles[i]), fmt_double(y[i], (styles[i] + 1) % 5)]
        cols = [None] * 4
        for k, pos in enumerate(order):
            cols[pos] = f[k]
        if messy:
            if i % 7 == 0:
                cols[order[2]] = '"' + cols[order[2]] + '"'
            if i % 3 == 0:
                cols[order[0]] = '"' + cols[order[0]] + '"'
            if i % 11 == 0:  # Double.valueOf trims; Long.valueOf would throw
                cols[order[3]] = " " + cols[order[3]] + "  "
            sep = [delim if (i + j) % 5 else (" " + delim + "  ") for j in range(3)]
        else:
            sep = [delim] * 3
        line = cols[0] + sep[0] + cols[1] + sep[1] + cols[2] + sep[2] + cols[3]
        if messy and i % 13 == 0:
            line += delim + "extra"
        lines.append(line)
    nl = "\r\n" if crlf else "\n"
    text = nl.join(lines) + (nl if trailing_newline else "")
    # the values a Java parser produces (Double.valueOf is correctly rounded, like float())
    px = np.array([float(fmt_double(v, s)) for v, s in zip(x, styles)])
    py = np.array([float(fmt_double(v, (s + 1) % 5)) for v, s in zip(y, styles)])
    return text.encode(), px, py, (obj_txt if string_objids else obj.astype(np.int64)), ts.astype(np.int64)
