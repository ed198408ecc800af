#!/usr/bin/env python3
"""Phase timestamps of the kNN pipeline (trace build: `make trace`, GF_TRACE).  Prints the
median per-phase durations over a run of continuous-query windows, hint on and off.
Timestamps: 100 MHz wall clock (10 ns ticks) written by thread 0 of the select kernel.
POLY=1: the polygon-query plan of `bench.py --workload polyknn` (0.02-degree square around the
query point; the sample / scan timestamps then do not apply)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GF_LIB_PATH", os.path.join(ROOT, "build", "libgeoflink_hip_trace.so"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import spatialflink_amd as sf  # noqa: E402
from spatialflink_amd import _lib  # noqa: E402

BEIJING = (115.5, 117.6, 39.6, 41.1)
Q = (116.414899, 39.920374)


def main():
    n, k, W, reps = 10_000_000, int(os.environ.get("K", "50")), 4, 40
    torch.cuda.set_device(0)
    grid = sf.UniformGrid(500, *BEIJING)
    wins = []
    for j in range(W):
        x, y = sf.synthetic_uniform(42 + j, n, *BEIJING[:4])
        wins.append(sf.PointWindow.from_numpy(x, y, np.arange(n, dtype=np.int64), device=0))
    if os.environ.get("POLY") == "1":
        h = 0.01
        ring = [(Q[0] - h, Q[1] - h), (Q[0] + h, Q[1] - h), (Q[0] + h, Q[1] + h), (Q[0] - h, Q[1] + h),
                (Q[0] - h, Q[1] - h)]
        op = sf.PointPolygonKNNQuery(sf.QueryConfiguration(sf.QueryType.WindowBased), grid)
        ctx, plan = op.plan(0, sf.Polygon([ring], grid), 0.5, k)
    else:
        op = sf.PointPointKNNQuery(sf.QueryConfiguration(sf.QueryType.WindowBased), grid)
        q = sf.Point("q", Q[0], Q[1], 0, grid)
        ctx, plan = op.plan(0, q, 0.5, k)
    L = _lib.lib()
    rb = L.gf_knn_result_bytes(k)
    stride = rb + 128
    # records (and the timestamps after them) in device memory: a store to mapped host memory
    # holds every later barrier for a PCIe round trip (s_waitcnt vmcnt(0) counts stores)
    dbuf = torch.zeros(stride * reps, dtype=torch.uint8, device="cuda")
    base = C.c_void_p(dbuf.data_ptr())
    buf = np.zeros(stride * reps, np.uint8)
    pts = [w.c_struct() for w in wins]
    names = ["load+zero", "hist", "binsearch", "compact", "sort+dedupe", "tail"]
    for hint in (1, 0):
        L.gf_knn_plan_set_hint(plan, hint)
        for i in range(8):
            L.gf_knn_enqueue(plan, C.byref(pts[i % W]), C.c_void_p(base.value + (i % reps) * stride))
        torch.cuda.synchronize()
        dbuf.zero_()
        torch.cuda.synchronize()
        for i in range(reps):
            L.gf_knn_enqueue(plan, C.byref(pts[i % W]), C.c_void_p(base.value + i * stride))
        L.gf_knn_plan_flush(plan)
        torch.cuda.synchronize()
        buf[:] = dbuf.cpu().numpy()
        rows = []
        for i in range(1, reps):
            tr = np.frombuffer(buf[i * stride + rb: i * stride + rb + 96].tobytes(), np.uint64).astype(np.int64)
            prev = np.frombuffer(buf[(i - 1) * stride + rb: (i - 1) * stride + rb + 96].tobytes(), np.uint64)
            prev = prev.astype(np.int64)
            t = tr[:7]
            row = [(t[j + 1] - t[j]) / 100.0 for j in range(6) if t[j + 1] and t[j]]
            row += [(tr[10] - tr[9]) / 100.0,   # sample start -> scan first block start
                    (tr[11] - tr[10]) / 100.0,  # scan span
                    (tr[0] - tr[11]) / 100.0,   # scan last block end -> select start
                    (t[6] - t[0]) / 100.0,      # select body
                    (tr[9] - prev[6]) / 100.0,  # previous select tail -> this sample start
                    float(tr[8])]
            rows.append(row)
        m = np.median(np.array([r for r in rows if len(r) == 12]), axis=0) if rows else None
        print(f"hint={hint} k={k}: median over {len(rows)} windows (us)")
        if m is not None:
            for nm, v in zip(names + ["sample->scan start", "scan span", "scan end->select start", "select body",
                                      "prev select->sample", "survivors cnt"], m):
                print(f"  {nm:24s} {v:8.2f}")


if __name__ == "__main__":
    main()
