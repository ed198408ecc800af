"""Single-GPU throughput of the other SURVEY.md §8 configurations (run through
`python bench.py --workload range|ppoly|join`); the default bench line stays kNN C2.

  range  C1: point-point range, 100x100 grid, 1M points per window, one query point, r = 0.5
         (and --radius), plus the same at 10M points per window.
  ppoly  C3: point-polygon range, the 1000 query polygons of generateQueryPolygons(1000, 115.5,
         39.6, 117.6, 41.1) (HelperClass.java:387-439), r = 0.001, 10M points per window.
  join   C4: point-point join, 10M ordinary x 1M query points, 1000x1000 grid, r = 0.001.

Each prints one JSON line with value = points/s over the timed windows (device-resident, a ring
of distinct windows), the dominant kernel's HIP-event time and its algorithmic bytes.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BEIJING = (115.5, 117.6, 39.6, 41.1)
QPOINT = (116.414899, 39.920374)
HBM_PEAK_GBS = 8000.0


def _windows(sf, n, count, seed0, dev=0):
    wins = []
    for j in range(count):
        x, y = sf.synthetic_uniform(seed0 + j, n, *BEIJING)
        wins.append((x, y, sf.PointWindow.from_numpy(x, y, np.arange(n, dtype=np.int64), device=dev)))
    return wins


def _line(workload, value, unit, steps, warmup, elapsed, kernel, bytes_per_launch, avg_s, extra):
    achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else None
    d = {"metric": f"points/sec per window ({workload})", "value": round(value, 1), "unit": unit, "n_gpus": 1,
         "steps": steps, "warmup": warmup, "ms_per_step": round(1000.0 * elapsed / steps, 4),
         "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
         "data": "synthetic: java.util.Random-compatible uniform points, Beijing bounds, device-resident",
         "roofline": {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1) if achieved else None,
                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                      "traffic": None, "bytes_per_launch": bytes_per_launch, "avg_launch_us": round(avg_s * 1e6, 2)}}
    d.update(extra)
    print(json.dumps(d), flush=True)


def bench_range(args, polygons=False):
    import torch

    import spatialflink_amd as sf
    from spatialflink_amd import _lib

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    L = _lib.lib()
    sizes = [args.points] if args.points else ([10_000_000] if polygons else [1_000_000, 10_000_000])
    sweep = [int(b) for b in str(args.range_blocks).split(",")]
    dsweep = [int(b) for b in str(args.range_defer).split(",")]
    for n, blocks, dmode in [(n, b, d) for n in sizes for b in sweep for d in dsweep]:
        grid_n = 500 if polygons else 100
        grid = sf.UniformGrid(grid_n, *BEIJING)
        og = O.grid(grid_n, *BEIJING)
        nwin = 4
        wins = _windows(sf, n, nwin, 7)
        conf = sf.QueryConfiguration(sf.QueryType.WindowBased)
        ctx = _lib.context(0)
        r = 0.001 if polygons else args.radius
        if polygons:
            raw = O.generate_query_polygons(1000, BEIJING[0], BEIJING[2], BEIJING[1], BEIJING[3])
            polys = [sf.Polygon(rings, grid) for rings in raw]
            ps = sf.PolygonSet(polys)
            cs = ps.c_struct()
            h = C.c_void_p()
            _lib.check(L.gf_range_ppoly_plan_create(ctx.handle, C.byref(grid.c_grid), C.byref(cs), r, 0, 0,
                                                    C.byref(h)), ctx.handle, "plan")
        else:
            qx = np.array([QPOINT[0]]); qy = np.array([QPOINT[1]])
            h = C.c_void_p()
            _lib.check(L.gf_range_pp_plan_create(ctx.handle, C.byref(grid.c_grid), qx.ctypes.data, qy.ctypes.data, 1,
                                                 r, 0, 0, C.byref(h)), ctx.handle, "plan")
        _lib.check(L.gf_range_plan_set_tuning(h, blocks, dmode), ctx.handle, "tuning")
        cells = [C.c_int64() for _ in range(4)]
        _lib.check(L.gf_range_plan_stats(h, *[C.byref(c) for c in cells]), ctx.handle, "stats")
        words = (n + 63) // 64
        bitmaps = torch.empty(nwin, words, dtype=torch.int64, device="cuda")
        counts = torch.zeros(nwin, 2, dtype=torch.int64, device="cuda")
        pts = [w[2].c_struct() for w in wins]

        def step(i):
            j = i % nwin
            st = L.gf_range_run(h, C.byref(pts[j]), bitmaps[j].data_ptr(), None, counts[j].data_ptr())
            if st:
                _lib.check(st, ctx.handle, "gf_range_run")

        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        ctx.set_timing_period(5)
        ctx.set_timing((1 << _lib.K_RANGE_SCAN) | (1 << _lib.K_RANGE_TEST))
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        ms, cnt = ctx.timing(_lib.K_RANGE_SCAN)
        tms, tcnt = ctx.timing(_lib.K_RANGE_TEST)
        ctx.set_timing(0)
        ctx.set_timing_period(1)
        # parity spot check of window 0 against the oracle: range results are per point, so the
        # first min(n, 1M) points of the window are checked against the oracle run on them alone
        hits = int(counts[0, 0].item())
        m = min(n, 1_000_000)
        x, y, _ = wins[0]
        exp = (O.range_ppoly(og, x[:m], y[:m], O.Polygons(raw), r) if polygons
               else O.range_pp(og, x[:m], y[:m], [QPOINT[0]], [QPOINT[1]], r))
        got = sf.spatialOperators.bitmap_indices(ctx, bitmaps[0], n).astype(np.int64)
        verified = bool(np.array_equal(got[got < m], exp))
        L.gf_range_plan_destroy(h)
        avg_scan = ms / 1000.0 / max(cnt, 1)
        avg_test = tms / 1000.0 / tcnt if tcnt else 0.0
        avg = avg_scan + avg_test
        wl = (f"ppoly_{len(polys)}polys_r{r}_{n // 1_000_000}Mpts_grid{grid_n}" if polygons
              else f"range_pp_r{r}_{n // 1_000_000}Mpts_grid{grid_n}")
        _line("point-polygon range" if polygons else "point-point range", n * args.steps / elapsed, "points/s",
              args.steps, args.warmup, elapsed,
              "range_kernel + range_test_kernel" if tcnt else "range_kernel", 16.0 * n + n / 8.0, avg,
              {"config": {"workload": wl, "points_per_window": n, "grid": grid_n, "radius": r,
                          "hits_window0": hits, "scan_blocks": blocks, "defer_mode": dmode,
                          "cells_none_candidate_guaranteed_inside": [c.value for c in cells]},
               "breakdown": {"scan_us": round(avg_scan * 1e6, 2), "test_us": round(avg_test * 1e6, 2)},
               "verified_vs_oracle": verified, "verified_sample": f"first {m} points of window 0"})


def bench_join(args):
    import torch

    import spatialflink_amd as sf
    from spatialflink_amd import _lib

    L = _lib.lib()
    no = args.points or 10_000_000
    nq = max(1, no // 10)
    grid = sf.UniformGrid(1000, *BEIJING)
    ctx = _lib.context(0)
    ow = _windows(sf, no, 2, 11)
    qw = _windows(sf, nq, 2, 21)
    r = 0.001
    cap = 4 * (no + nq)
    pairs = torch.empty(2 * cap, dtype=torch.int32, device="cuda")
    npairs = C.c_int64()
    po = [w[2].c_struct() for w in ow]
    pq = [w[2].c_struct() for w in qw]

    def step(i):
        _lib.check(L.gf_join_pp(ctx.handle, C.byref(grid.c_grid), C.byref(grid.c_grid), C.byref(po[i % 2]),
                                C.byref(pq[i % 2]), r, 0, 0, pairs.data_ptr(), cap, C.byref(npairs)),
                   ctx.handle, "gf_join_pp")

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    ctx.set_timing((1 << _lib.K_JOIN_PROBE) | (1 << _lib.K_JOIN_BUCKET))
    t0 = time.perf_counter()
    total_pairs = 0
    for i in range(args.steps):
        step(i)
        total_pairs += npairs.value
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms, cnt = ctx.timing(_lib.K_JOIN_PROBE)
    bms, bcnt = ctx.timing(_lib.K_JOIN_BUCKET)
    ctx.set_timing(0)
    avg = ms / 1000.0 / max(cnt, 1)
    pp = total_pairs / args.steps
    _line("point-point join", (no + nq) * args.steps / elapsed, "points/s", args.steps, args.warmup, elapsed,
          "join_probe (count + write passes, per launch)", 16.0 * no + 8.0 * pp / 2, avg,
          {"config": {"workload": f"join_pp_{no // 1_000_000}Mx{nq / 1e6:g}M_r{r}_grid1000", "ordinary": no,
                      "query": nq, "radius": r, "pairs_per_window": pp},
           "breakdown": {"probe_us_per_launch": round(avg * 1e6, 2), "probe_launches_per_window": cnt / args.steps,
                         "bucket_us_per_launch": round(bms * 1000.0 / max(bcnt, 1), 2),
                         "bucket_launches_per_window": bcnt / args.steps},
           "pairs_per_s": round(pp * args.steps / elapsed, 1)})


def run(args):
    if args.workload in ("range", "ppoly"):
        bench_range(args, polygons=args.workload == "ppoly")
    elif args.workload == "join":
        bench_join(args)
    else:
        raise SystemExit(f"unknown workload {args.workload}")
