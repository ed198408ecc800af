#!/usr/bin/env python3
"""Grid sweep for the fused continuous-query kNN kernel (pipeline depth 2) over a ring of 4
distinct 10M-point windows (640 MB, beyond the 256 MB Infinity Cache).  Per variant: wall
time per window over 60 windows (one sync at the end) and the HIP-event average of the fused
kernel (every 4th launch timed)."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import spatialflink_amd as sf  # noqa: E402
from spatialflink_amd import _lib  # noqa: E402

B = (115.5, 117.6, 39.6, 41.1)
Q = (116.414899, 39.920374)
N = 10_000_000
torch.cuda.set_device(0)
wins = []
for j in range(4):
    x, y = sf.synthetic_uniform(42 + j, N, *B)
    wins.append(sf.PointWindow.from_numpy(x, y, np.arange(N, dtype=np.int64)))
g = sf.UniformGrid(500, *B)
op = sf.PointPointKNNQuery(sf.QueryConfiguration(sf.QueryType.WindowBased), g)
q = sf.Point("q", *Q, 0, g)
ctx, plan = op.plan(0, q, 0.5, 50)
L = _lib.lib()
L.gf_knn_plan_set_pipeline(plan, 2)
rec = sf.PinnedRecords(64, 50)
pts = [w.c_struct() for w in wins]
refs = [C.byref(p) for p in pts]
variants = [(b, nt) for b in (256, 512, 768, 1024, 1280, 1536, 2048, 3072) for nt in (1, 0)]
res = {v: [] for v in variants}
for rnd in range(3):
    for v in variants:
        b, nt = v
        L.gf_knn_plan_set_tuning(plan, b, 1, nt)
        for i in range(6):
            L.gf_knn_enqueue(plan, refs[i % 4], rec.ptr(i))
        L.gf_knn_plan_flush(plan)
        torch.cuda.synchronize()
        ctx.set_timing_period(4)
        ctx.set_timing(1 << _lib.K_KNN_SCAN)
        t = time.perf_counter()
        for i in range(60):
            L.gf_knn_enqueue(plan, refs[i % 4], rec.ptr(i))
        L.gf_knn_plan_flush(plan)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) / 60 * 1e6
        ms, n = ctx.timing(_lib.K_KNN_SCAN)
        ctx.set_timing(0)
        res[v].append((wall, 1000 * ms / max(n, 1)))
        for i in range(60):
            assert rec.decode(i)[0] == 0
print(f"{'blocks':>6} {'nt':>2} | {'wall us':>8} {'Gpts/s':>7} | {'kernel us':>9} {'GB/s':>7}")
for v in variants:
    wall = min(r[0] for r in res[v])
    kern = min(r[1] for r in res[v])
    print(f"{v[0]:>6} {v[1]:>2} | {wall:8.2f} {N / wall / 1e3:7.1f} | {kern:9.2f} {16.0 * N / kern / 1e3:7.0f}")
