"""debug: per-window record status and idx offsets of the sliding engine vs the oracle"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import oracle as O
import spatialflink_amd as sf
from spatialflink_amd.spatialOperators import decode_knn_record
from test_gpu_sliding import make_stream, batches, expected_windows
BEIJING = (115.5, 117.6, 39.6, 41.1); QPOINT = (116.414899, 39.920374)
O.build()
size, slide, k, depth, n = 3000, 1000, 50, 2, 900_000
g = sf.UniformGrid(500, *BEIJING); og = O.grid(500, *BEIJING)
q = sf.Point("q", *QPOINT, 0, g)
x, y, obj, ts = make_stream(O, size + slide + k, n, 10_000, 24_000, gap=(15_200, 17_900))
op = sf.SlidingKNNQuery(sf.QueryConfiguration(sf.QueryType.WindowBased), g, q, 0.5, k, size_ms=size, slide_ms=slide,
                        pipeline=depth)
orig = op.results
def results():
    import torch
    torch.cuda.synchronize()
    for end, slot, first in (op.closed[:-1] if op.pending else op.closed):
        st, *_ = decode_knn_record(op.records.raw(slot), k)
        print("window end", end, "slot", slot, "first", first, "status", st, "base", op.panes.get(first, (0, None))[1])
    return orig()
got = []
for b in batches(sf, x, y, obj, ts, size):
    op.push(b)
    got += results()
op.flush()
got += results()
for r in got:
    m = (ts >= r.windowStart) & (ts < r.windowEnd)
    st, eo, ed, ei = O.knn(og, x[m], y[m], obj[m], QPOINT[0], QPOINT[1], 0.5, k)
    print(r.windowStart, r.windowEnd, "objOK", np.array_equal(r.objID, eo), "idx diffs", np.unique(ei - r.idx)[:5],
          "before", np.count_nonzero(ts < r.windowStart))
print("pane counts", np.bincount(ts // 1000)[10:])
