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


def make_csv(n, seed=0, delim=",", messy=False, order=(0, 1, 2, 3), crlf=False, trailing_newline=True):
    """-> (bytes, x, y, objID, ts): the exact values are those a correct parser must return."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(115.5, 117.6, n)
    y = rng.uniform(39.6, 41.1, n)
    obj = rng.integers(-10**12, 10**12, n)
    ts = rng.integers(0, 2 * 10**12, n)
    styles = rng.integers(0, 5, n) if messy else np.zeros(n, np.int64)
    lines = []
    for i in range(n):
        f = [str(int(obj[i])), str(int(ts[i])), fmt_double(x[i], styles[i]), fmt_double(y[i], (styles[i] + 1) % 5)]
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
    return text.encode(), px, py, obj.astype(np.int64), ts.astype(np.int64)
