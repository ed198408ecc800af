#!/usr/bin/env python3
"""Tuning sweep (one process, interleaved rounds): kNN scan-kernel grid / unroll / nontemporal
variants on a 10M-point window, next to a pure read probe of the same arrays.  Prints a table
of average kernel times (HIP events on the launch stream) and effective GB/s at 16 B/point."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import spatialflink_amd as sf  # noqa: E402
from spatialflink_amd import _lib  # noqa: E402

B = (115.5, 117.6, 39.6, 41.1)
Q = (116.414899, 39.920374)
N = int(os.environ.get("TUNE_N", 10_000_000))

torch.cuda.set_device(0)
x, y = sf.synthetic_uniform(42, N, *B)
w = sf.PointWindow.from_numpy(x, y, np.arange(N, dtype=np.int64))
g = sf.UniformGrid(500, *B)
conf = sf.QueryConfiguration(sf.QueryType.WindowBased)
q = sf.Point("q", *Q, 0, g)
op = sf.PointPointKNNQuery(conf, g)
ctx, plan = op.plan(0, q, 0.5, 50)
rec = torch.zeros(sf.spatialOperators.knn_record_bytes(50), dtype=torch.uint8, device="cuda")

probe = C.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
probe.hbm_probe.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]

variants = [(b, u, nt) for b in (1024, 2048, 4096, 8192) for u in (1, 2, 4, 8) for nt in (0, 1)]
res = {v: [] for v in variants}
pres = {v: [] for v in variants}
MB = 16.0 * N / 1e6
for rnd in range(3):
    for v in variants:
        b, u, nt = v
        _lib.check(_lib.lib().gf_knn_plan_set_tuning(plan, b, u, nt), ctx.handle, "tune")
        ctx.set_timing(1 << _lib.K_KNN_SCAN)
        for _ in range(10):
            op.enqueue(w, q, 0.5, 50, rec)
        ms, n = ctx.timing(_lib.K_KNN_SCAN)
        ctx.set_timing(0)
        res[v].append(ms / n)
        f = C.c_float()
        probe.hbm_probe(w.x.data_ptr(), w.y.data_ptr(), N // 2, b, u, nt, 10, C.byref(f))
        pres[v].append(f.value)
ctx.set_timing((1 << _lib.K_KNN_SAMPLE) | (1 << _lib.K_KNN_SELECT))
_lib.check(_lib.lib().gf_knn_plan_set_tuning(plan, 0, 4, 1), ctx.handle, "tune")
for _ in range(20):
    op.enqueue(w, q, 0.5, 50, rec)
smp = ctx.timing(_lib.K_KNN_SAMPLE)
sel = ctx.timing(_lib.K_KNN_SELECT)
print(f"N={N}  sample {1000*smp[0]/smp[1]:.2f} us  select {1000*sel[0]/sel[1]:.2f} us")
print(f"{'blocks':>6} {'U':>2} {'nt':>2} | {'scan us':>8} {'GB/s':>7} | {'probe us':>8} {'GB/s':>7}")
for v in variants:
    s = min(res[v]); p = min(pres[v])
    print(f"{v[0]:>6} {v[1]:>2} {v[2]:>2} | {1000*s:8.2f} {MB/s:7.0f} | {1000*p:8.2f} {MB/p:7.0f}")
