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


def _dist(args):
    """One process per GPU (torchrun env): (world, rank, device index).  Weak scaling: every
    rank holds the configuration's per-GPU share of points in its cell-column band."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local % torch.cuda.device_count())
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.cuda.current_device()


def _sync(world):
    import torch
    import torch.distributed as dist

    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()


def _reduce(v, world, args, dev, op="max"):
    """max (elapsed) / min (verified flags) over ranks."""
    if world == 1:
        return v
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(v)], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.MIN)
    return float(t.item())


def _reduce_sum(v, world, args, dev):
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(v)], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
    dist.all_reduce(t)
    return float(t.item())


def _host_threads():
    """This process's CPU share (OMP_NUM_THREADS on the GPU box, else every core), the machine's
    core count and CPU model."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    nproc, model = O.host_cpu()
    return min(nproc, int(os.environ.get("OMP_NUM_THREADS") or nproc)), nproc, model


def _timed(fn, budget):
    reps, t = 0, time.perf_counter()
    while True:
        out = fn()
        reps += 1
        el = time.perf_counter() - t
        if el >= budget:
            return reps, el, out


def _cpu_lines(args, unit, lines, check):
    """SURVEY.md 8(d) CPU baselines of a workload line, in the same run (rank 0, N = 1):
      value           the reference-shaped operator on every thread of this process's CPU share,
                      shaped as Flink runs it with that parallelism (conf/geoflink-conf.yml:55)
      single_thread   the same operator restated serially (1 thread)
      optimized_scan  an optimised OpenMP C line on the same threads (when there is one)
    lines: {"mt": (units per rep, fn(T), sample), "single": (...), "omp": (...) or None};
    check(results by name) -> every line's result equals the others' and the GPU's."""
    T, nproc, model = _host_threads()
    budget = max(1.0, args.cpu_seconds / 3.0)
    res, rate, samp = {}, {}, {}
    for name, spec in lines.items():
        if spec is None:
            continue
        units, fn, sample = spec
        reps, el, out = _timed(lambda: fn(1 if name == "single" else T), budget)
        res[name], rate[name] = out, reps * units / el
        samp[name] = f"{sample} x {reps} ({el:.1f}s)"
    ok = bool(check(res))
    d = {"value": round(rate["mt"], 1), "unit": unit, "cores": T, "kind": "port", "nproc": nproc, "cpu_model": model,
         "threads_note": "threads = this process's CPU share on the GPU box (OMP_NUM_THREADS), of nproc",
         "sample": samp["mt"] + ": the reference-shaped operator (C restatement) with Flink parallelism = threads",
         "results_equal_gpu": ok,
         "single_thread": {"value": round(rate["single"], 1), "unit": unit, "cores": 1, "kind": "port",
                           "sample": samp["single"] + ": the same operator, 1 thread"}}
    if "omp" in rate:
        d["optimized_scan"] = {"value": round(rate["omp"], 1), "unit": unit, "cores": T, "kind": "port",
                               "sample": samp["omp"] + ": optimised OpenMP C (integer cells, per-thread outputs)"}
    return d


def _pair_digest_dev(pairs, m: int) -> int:
    """oracle.pair_digest of the first m device pairs (uint32 pairs viewed as int32) computed on the
    device in chunks: sum mod 2^64 of fmix64(p << 32 | q) (torch int64 arithmetic wraps; logical
    right shifts by masking)."""
    import torch

    c1, c2 = 0xff51afd7ed558ccd - (1 << 64), 0xc4ceb9fe1a85ec53 - (1 << 64)
    mask33 = (1 << 31) - 1
    total = torch.zeros((), dtype=torch.int64, device=pairs.device)
    v = pairs[: 2 * m].view(-1, 2)
    for a in range(0, m, 1 << 27):
        blk = v[a:a + (1 << 27)].to(torch.int64) & 0xffffffff
        k = (blk[:, 0] << 32) | blk[:, 1]
        k = k ^ ((k >> 33) & mask33)
        k = k * c1
        k = k ^ ((k >> 33) & mask33)
        k = k * c2
        k = k ^ ((k >> 33) & mask33)
        total += k.sum()
    return int(total.item()) & ((1 << 64) - 1)


def _band(sf, grid, grid_n, world, rank):
    """x range of this rank's cell-column band (the whole grid at N = 1)."""
    from spatialflink_amd import sharding

    if world == 1:
        return BEIJING[0], BEIJING[1]
    lo, hi = sharding.column_bands(grid_n, world)[rank]
    return sharding.band_x_range(grid, lo, hi)


# --clustered: the BASELINE.md section 3 variant -- 80% of the points in 8 Gaussian hot spots
# (sigma 0.01 deg), the first on the query point, the other 7 fixed (the same for every window
# and both join sides, so the hot spots of the two sides overlap)
CLUSTERED = False


def hot_spots():
    r = np.random.default_rng(2024)
    return [QPOINT] + [(r.uniform(BEIJING[0], BEIJING[1]), r.uniform(BEIJING[2], BEIJING[3])) for _ in range(7)]


def gen_points(sf, seed, n, xlo, xhi):
    if not CLUSTERED:
        return sf.synthetic_uniform(seed, n, xlo, xhi, BEIJING[2], BEIJING[3])
    cs = [c for c in hot_spots() if xlo <= c[0] < xhi] or None
    return sf.synthetic_clustered(seed, n, xlo, xhi, BEIJING[2], BEIJING[3], centers=cs, n_centers=len(cs or [0]) or 1)


def data_desc():
    return ("synthetic: clustered -- 80% in 8 Gaussian hot spots (sigma 0.01 deg, one on the query point), 20% "
            "uniform, Beijing bounds, device-resident" if CLUSTERED else
            "synthetic: java.util.Random-compatible uniform points, Beijing bounds, device-resident")


def _windows(sf, n, count, seed0, dev=0, xr=None):
    wins = []
    xlo, xhi = xr or (BEIJING[0], BEIJING[1])
    for j in range(count):
        x, y = gen_points(sf, seed0 + j, n, xlo, xhi)
        wins.append((x, y, sf.PointWindow.from_numpy(x, y, np.arange(n, dtype=np.int64), device=dev)))
    return wins


def _line(workload, value, unit, steps, warmup, elapsed, kernel, bytes_per_launch, avg_s, extra, rank=0):
    if rank != 0:
        return
    achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else None
    d = {"metric": f"points/sec per window ({workload})", "value": round(value, 1), "unit": unit, "n_gpus": 1,
         "steps": steps, "warmup": warmup, "ms_per_step": round(1000.0 * elapsed / steps, 6),
         "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
         "data": data_desc(),
         "roofline": {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1) if achieved else None,
                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                      "traffic": None, "bytes_per_launch": bytes_per_launch, "avg_launch_us": round(avg_s * 1e6, 2)}}
    d.update(extra)
    from spatialflink_amd import _lib

    d["build"] = _lib.lib().gf_build_info().decode()
    print(json.dumps(d), flush=True)


def bench_range(args, polygons=False):
    """C1 / C3 range windows.  N > 1: weak scaling -- each rank holds the per-GPU window share
    (1M / 10M points) in its cell-column band and evaluates it with the full query set (query
    points / polygons replicated); hits need no exchange (each point is owned by one rank), so
    there is no collective in the data path.  value = points of all ranks / max elapsed.
    C3 at N > 1: the global window (N x 10M uniform points) is cut into bands balanced by WORK
    (sharding.work_bands: a point scan + 8 scans per point in a cell the plan tests exactly) --
    the 1000 polygons sit in the first ~37 of 500 columns, so even column bands would leave
    that work on rank 0 and the other ranks idle; a rank holds its band's share of the points."""
    import torch

    import spatialflink_amd as sf
    from spatialflink_amd import _lib

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    world, rank, dev = _dist(args)
    L = _lib.lib()
    sizes = [args.points] if args.points else ([10_000_000] if polygons else [1_000_000, 10_000_000])
    sweep = [int(b) for b in str(args.range_blocks).split(",")]
    dsweep = [int(b) for b in str(args.range_defer).split(",")]
    for n, blocks, dmode in [(n, b, d) for n in sizes for b in sweep for d in dsweep]:
        grid_n = 500 if polygons else 100
        grid = sf.UniformGrid(grid_n, *BEIJING)
        og = O.grid(grid_n, *BEIJING)
        # enough distinct windows that their x, y (16 B/point) exceed the 256 MB Infinity Cache:
        # every window is then read from HBM, not from the last window's residue
        r = 0.001 if polygons else args.radius
        band = _band(sf, grid, grid_n, world, rank)
        n_total = n * world
        if polygons:
            raw = O.generate_query_polygons(1000, BEIJING[0], BEIJING[2], BEIJING[1], BEIJING[3])
            if world > 1:
                from spatialflink_amd import sharding

                bb = [(min(p_[0] for p_ in rg[0]), min(p_[1] for p_ in rg[0]), max(p_[0] for p_ in rg[0]),
                       max(p_[1] for p_ in rg[0])) for rg in raw]
                per_cell = n_total / float(grid_n * grid_n)
                bands = sharding.work_bands(grid_n, world, np.full(grid_n, n_total / grid_n),
                                            sharding.candidate_cells_per_column(grid, bb, r) * per_cell,
                                            candidate_cost=8.0)
                lo, hi = bands[rank]
                band = sharding.band_x_range(grid, lo, hi)
                n = max(128, int(round(n_total * (hi - lo) / grid_n)))
        nwin = max(4, -(-384 * 2**20 // (16 * n)))
        ns_ = max(1, args.range_streams)
        batch = args.range_batch if args.range_batch > 0 else (16 if n <= 2_000_000 else 1)
        batch = max(1, min(batch, 16))
        # launch q (windows q*batch ..) runs on stream q % ns_; window j's buffers (points, bitmap,
        # index list) are reused by window j + nwin, which then runs on the same stream
        nwin = -(-nwin // (ns_ * batch)) * (ns_ * batch)
        wins = _windows(sf, n, nwin, 7 + 1000 * rank, dev, band)
        ctx = _lib.context(dev)
        if polygons:
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
        # --range-streams S: consecutive windows alternate over S contexts (each its own HIP stream
        # and plan), so window i+1's launch ramps up under window i's tail -- the range analogue
        # of the kNN plan's two-stream pipeline (windows are independent; results stay per window)
        ctxs, plans = [ctx], [h]
        for _ in range(max(1, args.range_streams) - 1):
            c2 = _lib.Context(dev)
            h2 = C.c_void_p()
            if polygons:
                _lib.check(L.gf_range_ppoly_plan_create(c2.handle, C.byref(grid.c_grid), C.byref(cs), r, 0, 0,
                                                        C.byref(h2)), c2.handle, "plan")
            else:
                _lib.check(L.gf_range_pp_plan_create(c2.handle, C.byref(grid.c_grid), qx.ctypes.data, qy.ctypes.data,
                                                     1, r, 0, 0, C.byref(h2)), c2.handle, "plan")
            _lib.check(L.gf_range_plan_set_tuning(h2, blocks, dmode), c2.handle, "tuning")
            ctxs.append(c2)
            plans.append(h2)
        cells = [C.c_int64() for _ in range(4)]
        _lib.check(L.gf_range_plan_stats(h, *[C.byref(c) for c in cells]), ctx.handle, "stats")
        words = (n + 63) // 64
        bitmaps = torch.empty(nwin, words, dtype=torch.int64, device=dev)
        counts = torch.zeros(nwin, 2, dtype=torch.int64, device=dev)
        # the step ends with the window's ascending index list on the device (what the Java
        # collector emits), produced by one async expansion launch after the scan
        idx = torch.empty(nwin, n, dtype=torch.int32, device=dev)  # window j's index list: idx[j]
        icount = torch.zeros(nwin, dtype=torch.int64, device=dev)
        pts = [w[2].c_struct() for w in wins]

        nstreams = len(plans)
        if batch > 1:  # windows i .. i+B-1 in one gf_range_run_batch (+ one index-list launch)
            P_ = C.c_void_p
            bms = [bitmaps[j].data_ptr() for j in range(nwin)]
            cnts = [counts[j].data_ptr() for j in range(nwin)]
            icnts = [icount[j].data_ptr() for j in range(nwin)]
            caps = (C.c_int64 * batch)(*([n] * batch))
            batch_args = []
            for g in range(nwin):  # group starting at window g (windows wrap around)
                js = [(g + u) % nwin for u in range(batch)]
                batch_args.append(((_lib.GfPoints * batch)(*[pts[j] for j in js]),
                                   (P_ * batch)(*[bms[j] for j in js]), (P_ * batch)(*[cnts[j] for j in js]),
                                   (P_ * batch)(*[idx[j].data_ptr() for j in js]),
                                   (P_ * batch)(*[icnts[j] for j in js])))

        def step(i):
            if batch > 1:
                if i % batch:
                    return
                pa, bm, ct, ix, ic = batch_args[i % nwin]
                c = ctxs[(i // batch) % nstreams].handle
                st = L.gf_range_run_batch(plans[(i // batch) % nstreams], batch, pa, bm, ct,
                                          None if args.no_indices else ix, caps, ic)
                if st:
                    _lib.check(st, c, "gf_range_run_batch")
                return
            j = i % nwin
            c = ctxs[i % nstreams].handle
            st = L.gf_range_run(plans[i % nstreams], C.byref(pts[j]), bitmaps[j].data_ptr(), None,
                                counts[j].data_ptr())
            if not st and not args.no_indices:
                st = L.gf_bitmap_to_indices_async(c, bitmaps[j].data_ptr(), n, idx[j].data_ptr(), n,
                                                  icount[j].data_ptr())
            if st:
                _lib.check(st, c, "gf_range_run")

        def sync_all():
            for c in ctxs:
                c.synchronize()
            torch.cuda.synchronize()

        steps = -(-args.steps // batch) * batch  # whole batches
        for i in range(-(-args.warmup // batch) * batch):
            step(i)
        sync_all()
        _sync(world)
        for c in ctxs:
            c.set_timing_period(5)
            c.set_timing((1 << _lib.K_RANGE_SCAN) | (1 << _lib.K_RANGE_TEST))
        _sync(world)
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        sync_all()
        elapsed = time.perf_counter() - t0
        if world > 1:
            import torch.distributed as dist

            dist.barrier()
        elapsed = _reduce(elapsed, world, args, dev)
        ms = cnt = tms = tcnt = 0
        for c in ctxs:
            a_ms, a_n = c.timing(_lib.K_RANGE_SCAN)
            b_ms, b_n = c.timing(_lib.K_RANGE_TEST)
            ms, cnt, tms, tcnt = ms + a_ms, cnt + a_n, tms + b_ms, tcnt + b_n
            c.set_timing(0)
            c.set_timing_period(1)
        # parity of window 0 against the oracle over the WHOLE window: the oracle's reference-shaped
        # evaluator on this process's threads (its Flink-parallelism form: the same per-point
        # results, sorted) -- on every rank, its shard's hits are exactly the oracle's hits of it
        hits = int(counts[0, 0].item())
        assert args.no_indices or int(icount[0].item()) == hits, "index list / counts disagree"
        m = n
        x, y, _ = wins[0]
        verified, cpu = None, None
        if not args.no_verify:
            T = max(1, _host_threads()[0] // max(world, 1))
            exp = (O.range_ppoly_mt(og, x, y, O.Polygons(raw), r, T) if polygons
                   else O.range_pp_mt(og, x, y, [QPOINT[0]], [QPOINT[1]], r, T))
            got = sf.spatialOperators.bitmap_indices(ctx, bitmaps[0], n).astype(np.int64)
            verified = bool(_reduce(float(np.array_equal(got, exp)), world, args, dev, op="min"))
            if world == 1 and not args.no_cpu_baseline:
                Pg = O.Polygons(raw) if polygons else None
                S = min(n, 200_000) if polygons else m  # the serial C3 operator tests 1000 polygons per point
                if polygons:
                    f1 = lambda T, k=S: O.range_ppoly(og, x[:k], y[:k], Pg, r)  # noqa: E731
                    fm = lambda T: O.range_ppoly_mt(og, x, y, Pg, r, T)  # noqa: E731
                    fo = lambda T: O.range_ppoly_mt(og, x, y, Pg, r, T, optimized=True)  # noqa: E731
                else:
                    f1 = lambda T, k=S: O.range_pp(og, x[:k], y[:k], [QPOINT[0]], [QPOINT[1]], r)  # noqa: E731
                    fm = lambda T: O.range_pp_mt(og, x, y, [QPOINT[0]], [QPOINT[1]], r, T)  # noqa: E731
                    fo = lambda T: O.range_pp_mt(og, x, y, [QPOINT[0]], [QPOINT[1]], r, T, optimized=True)  # noqa: E731
                cpu = _cpu_lines(args, "points/s", {
                    "mt": (n, fm, f"the whole {n}-point window 0"),
                    "single": (S, f1, f"first {S} points of window 0"),
                    "omp": (n, fo, f"the whole {n}-point window 0")},
                    lambda R: np.array_equal(R["mt"], got) and np.array_equal(R["omp"], got)
                    and np.array_equal(R["single"], got[got < S]))
        for hp in plans:
            L.gf_range_plan_destroy(hp)
        avg_scan = ms / 1000.0 / max(cnt, 1) / batch  # a batched launch evaluates `batch` windows
        avg_test = tms / 1000.0 / tcnt if tcnt else 0.0
        avg = avg_scan + avg_test
        # with windows in flight on several streams a launch's own duration counts shared time
        # more than once: the roofline then uses the sustained interval between windows
        basis = "bytes per window / average launch duration per window (one stream)"
        if nstreams > 1:
            avg = elapsed / steps
            basis = f"bytes per window / window interval ({nstreams} streams; includes host work)"
        wl = (f"ppoly_{len(polys)}polys_r{r}_{n // 1_000_000}Mpts_grid{grid_n}" if polygons
              else f"range_pp_r{r}_{n // 1_000_000}Mpts_grid{grid_n}")
        if world > 1:
            wl += f"_per_gpu_x{world}"
        n_all = int(_reduce_sum(float(n), world, args, dev)) if world > 1 else n
        _line("point-polygon range" if polygons else "point-point range", n_all * steps / elapsed,
              "points/s", steps, args.warmup, elapsed,
              "range_kernel + range_test_kernel" if tcnt else "range_kernel", 16.0 * n + n / 8.0 + 4.0 * hits, avg,
              {"n_gpus": world,
               "config": {"workload": wl, "points_per_window": n_all, "points_per_gpu": n, "grid": grid_n,
                          "radius": r, "hits_window0": hits, "scan_blocks": blocks, "defer_mode": dmode,
                          "windows_in_flight": nstreams, "distinct_windows": nwin,
                          "window_set_MB": round(16.0 * n * nwin / 2**20, 1),
                          "step": ("gf_range_run (bitmap + counts) + gf_bitmap_to_indices_async (index list)"
                                   if batch == 1 else f"gf_range_run_batch of {batch} windows (bitmaps + counts "
                                   "in one launch, index lists in one more); value counts every window"),
                          "windows_per_launch": batch,
                          "parallelism": f"cell-column shards x{world} (no collective)" + (
                              ", bands balanced by work (points + 8 x candidate-cell points)"
                              if polygons and world > 1 else ""),
                          "cells_none_candidate_guaranteed_inside": [c.value for c in cells]},
               "breakdown": {"scan_us": round(avg_scan * 1e6, 2), "test_us": round(avg_test * 1e6, 2),
                             "achieved_basis": basis},
               "verified_vs_oracle": verified,
               "verified_sample": f"the whole {m}-point window 0 on every rank (oracle on {_host_threads()[0] // max(world, 1)} threads)",
               **({"cpu_baseline": cpu} if cpu else {})},
              rank=rank)


def bench_join(args):
    """C4 join.  N > 1: weak scaling, grid-partitioned -- each rank holds 10M ordinary points of
    its cell-column band; the query side (1M per GPU, the same global set on every rank) is
    replicated with a c-column halo (sharding.join_query_halo), so every pair is produced once,
    by its ordinary point's owner, with no collective in the data path."""
    import torch

    import spatialflink_amd as sf
    from spatialflink_amd import _lib, sharding

    world, rank, dev = _dist(args)
    L = _lib.lib()
    no = args.points or 10_000_000
    nq = max(1, no // 10)
    grid_n = 1000
    grid = sf.UniformGrid(grid_n, *BEIJING)
    ctx = _lib.context(dev)
    if getattr(args, "join_stream", False):  # experiment: query side bucketed only, ordinary points streamed
        _lib.check(L.gf_ctx_set_flag(ctx.handle, _lib.FLAG_JOIN_STREAM, 1), ctx.handle, "flag")
    ow = _windows(sf, no, 2, 11 + 1000 * rank, dev, _band(sf, grid, grid_n, world, rank))
    r = 0.001
    if world == 1:
        qw = _windows(sf, nq, 2, 21, dev)
    else:
        band = sharding.column_bands(grid_n, world)[rank]
        c = int(np.ceil(r / grid.getCellLength()))
        qw = []
        for j in range(2):
            x, y = gen_points(sf, 21 + j, nq * world, BEIJING[0], BEIJING[1])
            keep = sharding.join_query_halo(np.floor((x - BEIJING[0]) / grid.getCellLength()), band, c)
            xs, ys = np.ascontiguousarray(x[keep]), np.ascontiguousarray(y[keep])
            qw.append((xs, ys, sf.PointWindow.from_numpy(xs, ys, np.flatnonzero(keep).astype(np.int64), device=dev)))
    nq_rank = len(qw[0][0])
    cap = 4 * (no + nq_rank)
    pairs = torch.empty(2 * cap, dtype=torch.int32, device=dev)
    npairs = C.c_int64()
    # windows in flight (--join-streams, default 2): consecutive windows alternate over contexts --
    # each its own stream, scratch, output buffer and region history -- so one window's kernels
    # fill the other's launch gaps and latency-bound phases (the kNN plan's depth 3, the range
    # bench's --range-streams); every window still runs its whole join
    nstreams = max(1, getattr(args, "join_streams", 2))
    ctxs = [ctx] + [_lib.Context(dev) for _ in range(nstreams - 1)]
    if getattr(args, "join_stream", False):
        for c_ in ctxs[1:]:
            _lib.check(L.gf_ctx_set_flag(c_.handle, _lib.FLAG_JOIN_STREAM, 1), c_.handle, "flag")
    po = [w[2].c_struct() for w in ow]
    pq = [w[2].c_struct() for w in qw]

    def step(i):
        _lib.check(L.gf_join_pp(ctx.handle, C.byref(grid.c_grid), C.byref(grid.c_grid), C.byref(po[i % 2]),
                                C.byref(pq[i % 2]), r, 0, 0, pairs.data_ptr(), cap, C.byref(npairs)),
                   ctx.handle, "gf_join_pp")

    # output capacity: sized from a counting call on each window (clustered inputs produce
    # hundreds of pairs per point in the hot spots), outside the timed region
    for i in range(2):
        st = L.gf_join_pp(ctx.handle, C.byref(grid.c_grid), C.byref(grid.c_grid), C.byref(po[i]), C.byref(pq[i]), r,
                          0, 0, None, 0, C.byref(npairs))
        if st not in (0, _lib.GF_ERR_CAPACITY):
            _lib.check(st, ctx.handle, "gf_join_pp (count)")
        if npairs.value > cap:
            cap = int(1.05 * npairs.value) + 1024
    if 2 * cap > pairs.numel():
        del pairs
        pairs = torch.empty(2 * cap, dtype=torch.int32, device=dev)
    outs = [pairs] + [torch.empty(2 * cap, dtype=torch.int32, device=dev) for _ in range(nstreams - 1)]
    for c_ in ctxs[1:]:  # each context's region history from a call on the same windows
        for i in range(2):
            L.gf_join_pp(c_.handle, C.byref(grid.c_grid), C.byref(grid.c_grid), C.byref(po[i]), C.byref(pq[i]), r,
                         0, 0, None, 0, C.byref(npairs))

    # default: gf_join_pp_async -- each window's launches queue behind the previous window (no
    # host wait for its pair count); the counts land in device memory, read after the final sync
    use_async = not getattr(args, "join_sync", False)
    totals = torch.zeros(max(args.steps, 1), dtype=torch.int64, device=dev)

    def step_async(i):
        c_ = ctxs[i % nstreams]
        _lib.check(L.gf_join_pp_async(c_.handle, C.byref(grid.c_grid), C.byref(grid.c_grid), C.byref(po[i % 2]),
                                      C.byref(pq[i % 2]), r, 0, 0, outs[i % nstreams].data_ptr(), cap,
                                      totals[i].data_ptr()), c_.handle, "gf_join_pp_async")

    for i in range(args.warmup):
        step(i)
    _sync(world)
    if use_async and nstreams > 1:  # the windows' inputs were produced before: no cross-stream waits
        torch.cuda.synchronize()
    for c_ in ctxs:
        c_.set_timing((1 << _lib.K_JOIN_PROBE) | (1 << _lib.K_JOIN_BUCKET))
    _sync(world)
    t0 = time.perf_counter()
    total_pairs = 0
    for i in range(args.steps):
        if use_async:
            step_async(i)
        else:
            step(i)
            total_pairs += npairs.value
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if use_async:
        counts = totals.cpu().numpy()
        if (counts > cap).any():
            raise RuntimeError("gf_join_pp_async: a window's pairs exceeded the buffer")
        total_pairs = int(counts.sum())
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    elapsed = _reduce(elapsed, world, args, dev)
    ms = cnt = bms = bcnt = 0
    for c_ in ctxs:  # each context times its own windows' launches (HIP events on its stream)
        m_, c1 = c_.timing(_lib.K_JOIN_PROBE)
        b_, c2 = c_.timing(_lib.K_JOIN_BUCKET)
        ms, cnt, bms, bcnt = ms + m_, cnt + c1, bms + b_, bcnt + c2
        c_.set_timing(0)
    avg = ms / 1000.0 / max(cnt, 1)
    pp = total_pairs / args.steps
    pp_all = pp if world == 1 else _reduce_sum(pp, world, args, dev)
    # parity (N = 1): EVERY pair of both windows (the whole 10M x 1M window, not a sample) against
    # the oracle's optimised OpenMP join, which the reference-shaped join pins on the first 1M
    # ordinary points of window 0; every timed async window's count == its window's synchronous
    # count.  CPU baseline on that 1M-point sample (pairs are per ordinary point), timed.
    verified, cpu = None, None
    if world == 1 and not args.no_verify:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        def sorted_pairs(a):
            return a[np.lexsort((a[:, 1], a[:, 0]))]

        og = O.grid(grid_n, *BEIJING)
        nthr = _host_threads()[0]
        verified = True
        digest_mode = False
        for wi in range(2):
            step(wi)
            if use_async:
                tc = totals[: args.steps].cpu().numpy()[wi::2]
                if not (tc == npairs.value).all():
                    raise RuntimeError(f"gf_join_pp_async counts {set(tc.tolist())} != gf_join_pp {npairs.value}")
            (x, y, _), (qx, qy, _) = ow[wi], qw[wi]
            if npairs.value > 200_000_000:  # (clustered: 2e9 pairs) count + order-free digest of every pair
                digest_mode = True
                ecnt, edg = O.join_pp_digest(og, x, y, qx, qy, r, nthr)
                verified = verified and ecnt == npairs.value and edg == _pair_digest_dev(pairs, npairs.value)
            else:
                got_w = sorted_pairs(pairs[: 2 * npairs.value].cpu().numpy().view(np.uint32).astype(np.int64)
                                     .reshape(-1, 2))
                exp_w = O.join_pp_mt(og, og, x, y, qx, qy, r, nthr, optimized=True)
                verified = verified and bool(np.array_equal(got_w, exp_w))
            if wi == 0:
                m = min(no, 1_000_000)
                g0 = pairs[: 2 * npairs.value].view(-1, 2)
                g0 = g0[g0[:, 0].to(torch.int64) < m].cpu().numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
                got_s = sorted_pairs(g0)
        (x, y, _), (qx, qy, _) = ow[0], qw[0]
        st, exp = O.join_pp(og, og, x[:m], y[:m], qx, qy, r)
        verified = verified and bool(st == 0 and np.array_equal(got_s, sorted_pairs(exp)))
        if not args.no_cpu_baseline:  # the first m ordinary points x the whole query window (pairs are per point)
            cpu = _cpu_lines(args, "points/s", {
                "mt": (m + len(qx), lambda T: O.join_pp_mt(og, og, x[:m], y[:m], qx, qy, r, T),
                       f"first {m} ordinary points of window 0 x the {len(qx)} query points"),
                "single": (m + len(qx), lambda T: sorted_pairs(O.join_pp(og, og, x[:m], y[:m], qx, qy, r)[1]),
                           f"first {m} ordinary points of window 0 x the {len(qx)} query points"),
                "omp": (m + len(qx), lambda T: O.join_pp_mt(og, og, x[:m], y[:m], qx, qy, r, T, optimized=True),
                        f"first {m} ordinary points of window 0 x the {len(qx)} query points")},
                lambda R: all(np.array_equal(R[k_], got_s) for k_ in ("mt", "single", "omp")))
    wl = f"join_pp_{no // 1_000_000}Mx{nq / 1e6:g}M_r{r}_grid1000" + (f"_per_gpu_x{world}" if world > 1 else "") + (
        "_clustered" if CLUSTERED else "")
    # roofline over the WHOLE window (every join kernel: both bucketings, probe, packing): the
    # algorithmic bytes are the two sides' xy read once and the pairs written once
    _line("point-point join", world * (no + nq) * args.steps / elapsed, "points/s", args.steps, args.warmup, elapsed,
          "window (query + ordinary row bucketing, join_row_probe, packing): xy of both sides in once, pairs out once",
          16.0 * (no + nq_rank) + 8.0 * pp, elapsed / args.steps,
          {"n_gpus": world,
           "config": {"workload": wl, "ordinary": no * world, "query": nq * world, "radius": r,
                      "pairs_per_window": pp_all, "query_per_rank_with_halo": nq_rank,
                      "window_api": (f"gf_join_pp_async, {nstreams} windows in flight (consecutive windows alternate over "
                                     f"{nstreams} contexts / streams; counts read after the final sync)")
                      if use_async else "gf_join_pp (pair count read back per window)",
                      "windows_in_flight": nstreams if use_async else 1,
                      "parallelism": f"cell-column shards x{world}, query halo c columns (no collective)"},
           "breakdown": {"probe_us_per_launch": round(avg * 1e6, 2), "probe_launches_per_window": cnt / args.steps,
                         "probe_GBps_row_bucketed_in_pairs_out": round((20.0 * no + 8.0 * pp) / avg / 1e9, 1) if avg > 0 else None,
                         "bucket_us_per_launch": round(bms * 1000.0 / max(bcnt, 1), 2),
                         "bucket_launches_per_window": bcnt / args.steps},
           "pairs_per_s": round(pp_all * args.steps / elapsed, 1), "verified_vs_oracle": verified,
           **({"verified_sample": ("whole window: " + ("the pair count and an order-free digest of every pair "
                                  "(sum of fmix64(p << 32 | q))" if digest_mode else "every pair") +
                                  " of both windows vs the oracle's OpenMP join; the pairs of the first 1M "
                                  "ordinary points of window 0 vs the reference-shaped join; every timed "
                                  "window's count == its window's")}
              if verified is not None else {}),
           **({"cpu_baseline": cpu} if cpu else {})}, rank=rank)


def bench_pjoin(args):
    """Point-polygon window join (PointPolygonJoinQuery): the C3 shapes --
    the 1000 generateQueryPolygons squares as the polygon side, 10M points per window, 500 x 500
    grid, r = 0.001.  A step = one window: scan (every point whose cell some polygon replicates
    to is queued) + count pass + write pass + the pair count read back (sync).  N > 1: weak
    scaling, points sharded by cell-column bands, polygons replicated, no collective."""
    import torch

    import spatialflink_amd as sf
    from spatialflink_amd import _lib

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    world, rank, dev = _dist(args)
    L = _lib.lib()
    n = args.points or 10_000_000
    grid_n = 500
    grid = sf.UniformGrid(grid_n, *BEIJING)
    og = O.grid(grid_n, *BEIJING)
    nwin = 4
    wins = _windows(sf, n, nwin, 17 + 1000 * rank, dev, _band(sf, grid, grid_n, world, rank))
    ctx = _lib.context(dev)
    r = 0.001
    raw = O.generate_query_polygons(1000, BEIJING[0], BEIJING[2], BEIJING[1], BEIJING[3])
    polys = [sf.Polygon(rings, grid) for rings in raw]
    ps = sf.PolygonSet(polys)
    cs = ps.c_struct()
    h = C.c_void_p()
    _lib.check(L.gf_join_ppoly_plan_create(ctx.handle, C.byref(grid.c_grid), C.byref(cs), r, 0, 0, C.byref(h)),
               ctx.handle, "plan")
    cap = max(1 << 20, n // 4)
    pairs = torch.empty(2 * cap, dtype=torch.int32, device=dev)
    npairs = C.c_int64()
    pts = [w[2].c_struct() for w in wins]
    counts = [0] * nwin

    def step(i):
        _lib.check(L.gf_join_ppoly_run(h, C.byref(grid.c_grid), C.byref(pts[i % nwin]), pairs.data_ptr(), cap,
                                       C.byref(npairs)), ctx.handle, "gf_join_ppoly_run")
        counts[i % nwin] = npairs.value

    for i in range(args.warmup):
        step(i)
    _sync(world)
    ctx.set_timing((1 << _lib.K_RANGE_SCAN) | (1 << _lib.K_RANGE_TEST))
    _sync(world)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    elapsed = _reduce(elapsed, world, args, dev)
    ms, cnt = ctx.timing(_lib.K_RANGE_SCAN)
    tms, tcnt = ctx.timing(_lib.K_RANGE_TEST)
    ctx.set_timing(0)
    verified, cpu = None, None
    if not args.no_verify:  # the WHOLE window 0 vs the oracle (its Flink-parallelism form, sorted pairs)
        step(0)
        torch.cuda.synchronize()
        got = pairs[: 2 * npairs.value].cpu().numpy().view(np.uint32).astype(np.int64).reshape(-1, 2)
        got = got[np.lexsort((got[:, 1], got[:, 0]))]
        x, y, _ = wins[0]
        Pg = O.Polygons(raw)
        T = max(1, _host_threads()[0] // max(world, 1))
        exp_arr = O.join_ppoly_mt(og, og, x, y, Pg, r, T)
        if world == 1 and not args.no_cpu_baseline:
            m = min(n, 1_000_000)

            def sorted_pairs(a_):
                return a_[np.lexsort((a_[:, 1], a_[:, 0]))]
            cpu = _cpu_lines(args, "points/s", {
                "mt": (n, lambda T_: O.join_ppoly_mt(og, og, x, y, Pg, r, T_),
                       f"the whole {n}-point window 0 x the 1000 polygons (polygons replicated to string keys, hash "
                       "join on gridID, JTS distance per co-located pair)"),
                "single": (m, lambda T_: sorted_pairs(O.join_ppoly(og, og, x[:m], y[:m], Pg, r)),
                           f"first {m} points of window 0 x the 1000 polygons")},
                lambda R: np.array_equal(R["mt"], exp_arr) and np.array_equal(R["single"], exp_arr[exp_arr[:, 0] < m]))
        verified = bool(_reduce(float(np.array_equal(got, exp_arr)), world, args, dev, op="min"))
    L.gf_range_plan_destroy(h)
    avg_scan = ms / 1000.0 / max(cnt, 1)
    avg_test = tms / 1000.0 / max(tcnt, 1)
    pp = float(np.mean(counts))
    wl = f"join_ppoly_{len(polys)}polys_r{r}_{n // 1_000_000}Mpts_grid{grid_n}" + (f"_per_gpu_x{world}" if world > 1 else "")
    _line("point-polygon join", world * n * args.steps / elapsed, "points/s", args.steps, args.warmup, elapsed,
          "range_kernel (join queue) + join_ppoly count/write", 16.0 * n + 8.0 * pp, avg_scan + avg_test,
          {"n_gpus": world,
           "config": {"workload": wl, "points_per_window": n * world, "points_per_gpu": n, "grid": grid_n, "radius": r,
                      "polygons": len(polys), "pairs_per_window_rank0": pp,
                      "parallelism": f"cell-column shards x{world} (no collective)"},
           "breakdown": {"scan_us": round(avg_scan * 1e6, 2), "count_write_us": round(avg_test * 1e6, 2)},
           "verified_vs_oracle": verified, "verified_sample": f"the whole {n}-point window 0 (every pair)",
           **({"cpu_baseline": cpu} if cpu else {})},
          rank=rank)


def bench_sliding(args):
    """C5: sliding-window kNN, k = 100, 1000 x 1000 grid, 100M points per window, size/slide = 2
    (panes of 50M points), r = 0.5 around the README query point.  A step = one slide: one pane
    pushed through the pane engine (one fused scan/select launch) and one window record merged
    from its two panes.  value = window points / s (each window holds 100M points; the
    reference re-evaluates all of them per window, the engine scans each pane once).  N > 1:
    strong scaling -- the window's points are split across ranks by cell-column bands, each
    rank runs its own pane engine on its band and the window records of B consecutive windows
    are all-gathered over RCCL and merged in one launch."""
    import torch
    import torch.distributed as dist

    import spatialflink_amd as sf
    from spatialflink_amd import _lib, sharding
    from spatialflink_amd.spatialOperators import knn_record_bytes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local % torch.cuda.device_count())
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    L = _lib.lib()
    k = args.k if args.k != 50 else 100
    grid_n = args.grid if args.grid != 500 else 1000
    window_pts = args.points or 100_000_000
    W = 2                                     # size / slide
    pane_pts = window_pts // W // world       # this rank's share of one pane
    pane_pts -= pane_pts % 2
    npanes = max(3, args.windows)             # distinct device-resident panes cycled
    grid = sf.UniformGrid(grid_n, *BEIJING)
    if world == 1:
        xlo, xhi = BEIJING[0], BEIJING[1]
    else:
        lo, hi = sharding.column_bands(grid_n, world)[rank]
        xlo, xhi = sharding.band_x_range(grid, lo, hi)
    t = time.perf_counter()
    panes, host = [], []
    for j in range(npanes):
        x, y = sf.synthetic_uniform(4242 + 1000 * rank + j, pane_pts, xlo, xhi, BEIJING[2], BEIJING[3])
        obj = np.arange(pane_pts, dtype=np.int64) + (rank * npanes + j) * pane_pts
        panes.append(sf.PointWindow.from_numpy(x, y, obj, device=dev))
        host.append((x, y, obj))
    torch.cuda.synchronize()
    print(f"[rank {rank}] {npanes} panes x {pane_pts} points generated+uploaded in {time.perf_counter() - t:.1f}s",
          file=sys.stderr, flush=True)
    conf = sf.QueryConfiguration(sf.QueryType.WindowBased)
    q = sf.Point("q", QPOINT[0], QPOINT[1], 0, grid)
    op = sf.PointPointKNNQuery(conf, grid)
    ctx, plan = op.plan(dev, q, args.radius, k)
    depth = min(args.pipeline, 2)  # the pane engine runs at depth <= 2
    _lib.check(L.gf_knn_plan_set_pipeline(plan, depth), ctx.handle, "pipeline")
    size_ms, slide_ms = 2000, 1000
    eng = C.c_void_p()
    _lib.check(L.gf_knn_sliding_create(plan, size_ms, slide_ms, C.byref(eng)), ctx.handle, "sliding")
    rb = knn_record_bytes(k)
    B = max(1, args.exchange_batch)
    total = args.warmup + args.steps
    recs = torch.zeros(total, rb, dtype=torch.uint8, device=dev)   # rank-local window records
    merged = sf.PinnedRecords(total, k) if world > 1 else None
    out = merged if world > 1 else sf.PinnedRecords(total, k)
    pts = [p.c_struct() for p in panes]
    closed, wend = C.c_int32(), C.c_int64()
    lag = 1 if depth == 2 else 0
    push = L.gf_knn_sliding_push

    comm, xdesc = sharding.open_comm(dev, args.dist_backend, args.exchange) if world > 1 else (None, None)

    def exchange(lo, hi):  # windows [lo, hi]: one all-gather + one merge launch
        if comm is not None:  # the C ABI's RCCL communicator (gf_knn_exchange_batch)
            comm.exchange_batch(recs[lo:hi + 1], k, out.ptr(lo), ctx=ctx)
        else:
            sharding.allgather_knn_records_batch(recs[lo:hi + 1], k, out.ptr(lo))

    def step(i, first):
        dst = recs[i].data_ptr() if world > 1 else out.ptr(i)
        st = push(eng, i, C.byref(pts[i % npanes]), C.c_void_p(dst), C.byref(closed), C.byref(wend))
        if st:
            _lib.check(st, ctx.handle, "gf_knn_sliding_push")
        if world > 1:
            c = i - lag
            if c >= first and (c - first) % B == B - 1:
                exchange(c - B + 1, c)

    def drain(first, last):
        _lib.check(L.gf_knn_sliding_flush(eng), ctx.handle, "flush")
        if world > 1:
            lo = first + ((last - first) // B) * B
            if lag or (last - first) % B != B - 1:
                exchange(lo, last)

    for i in range(args.warmup):
        step(i, 0)
    drain(0, args.warmup - 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ctx.set_timing_period(args.timing_period)
    ctx.set_timing((1 << _lib.K_KNN_SCAN) | (1 << _lib.K_KNN_MERGE))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.warmup, total):
        step(i, args.warmup)
    drain(args.warmup, total - 1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    scan_ms, scan_n = ctx.timing(_lib.K_KNN_SCAN)
    merge_ms, merge_n = ctx.timing(_lib.K_KNN_MERGE)
    ctx.set_timing(0)
    ctx.set_timing_period(1)
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # every timed window record is final (no fallback) and deterministic per distinct window
    # (engine idx = stream position; window i starts at pane i-1, position (i-1) * pane_pts)
    per = {}
    for i in range(max(1, args.warmup), total):
        st, o, d, ix = out.decode(i)
        assert st == 0, f"window {i} needed the exact fallback inside the timed region"
        key = ((i - 1) % npanes, i % npanes)
        rel = ix - (i - 1) * pane_pts
        if key in per:
            assert all(np.array_equal(u, v) for u, v in zip(per[key], (o, d, rel))), "non-deterministic"
        else:
            per[key] = (o, d, rel)

    # parity (N = 1): each distinct window == the same plan's whole-window evaluation of the two
    # panes concatenated (the reference's from-scratch evaluation; gf_knn_run is oracle-checked in
    # tests/), and the first window == the oracle; plus the from-scratch time for comparison
    verified, scratch_us = None, None
    if world == 1 and not args.no_verify:
        op2 = sf.PointPointKNNQuery(conf, grid)
        ctx2, plan2 = op2.plan(dev, q, args.radius, k)
        verified = True
        for (a, b), (o, d, ix) in sorted(per.items()):
            wa, wb = panes[a], panes[b]
            cat = sf.PointWindow(torch.cat([wa.x, wb.x]), torch.cat([wa.y, wb.y]), torch.cat([wa.objID, wb.objID]),
                                 torch.cat([wa.timeStampMillisec, wb.timeStampMillisec]))
            res = op2.run(cat, q, args.radius, k)
            verified &= bool(np.array_equal(res.objID, o) and np.array_equal(res.dist, d)
                             and np.array_equal(res.idx, ix))
            if scratch_us is None:  # the from-scratch alternative: one 100M-point evaluation per window
                _lib.check(L.gf_knn_plan_set_pipeline(plan2, args.pipeline), ctx2.handle, "pipeline")
                tmp = torch.zeros(8, rb, dtype=torch.uint8, device=dev)
                cs = cat.c_struct()
                for it in range(3):
                    L.gf_knn_enqueue(plan2, C.byref(cs), C.c_void_p(tmp[it].data_ptr()))
                L.gf_knn_plan_flush(plan2)
                torch.cuda.synchronize()
                ts_ = time.perf_counter()
                for it in range(8):
                    L.gf_knn_enqueue(plan2, C.byref(cs), C.c_void_p(tmp[it].data_ptr()))
                L.gf_knn_plan_flush(plan2)
                torch.cuda.synchronize()
                scratch_us = 1e6 * (time.perf_counter() - ts_) / 8
            del cat
        assert verified, "pane-merged windows differ from whole-window evaluation"
        if not args.no_verify:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O

            (a, b), (o, d, ix) = sorted(per.items())[0]
            X = np.concatenate([host[a][0], host[b][0]]); Y = np.concatenate([host[a][1], host[b][1]])
            OB = np.concatenate([host[a][2], host[b][2]])
            t = time.perf_counter()
            st, eo, ed, ei = O.knn(O.grid(grid_n, *BEIJING), X, Y, OB, QPOINT[0], QPOINT[1], args.radius, k)
            verified &= bool(st == 0 and np.array_equal(eo, o) and np.array_equal(ed, d) and np.array_equal(ei, ix))
            print(f"oracle check of one {len(X)}-point window: {verified} ({time.perf_counter() - t:.1f}s)",
                  file=sys.stderr, flush=True)
            assert verified, "pane-merged window differs from the oracle"
    if world > 1 and rank == 0 and not args.no_verify and window_pts <= 100_000_000:
        # the all-gathered, device-merged record of one window == the oracle on the union of
        # every rank's two panes (rank 0 regenerates the other bands from their seeds).  objIDs
        # are globally unique; idx is each rank's own stream position, so it is not compared.
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        (a, b), (o, d, ix) = sorted(per.items())[0]
        xs, ys, obs = [], [], []
        for r_ in range(world):
            blo, bhi = sharding.column_bands(grid_n, world)[r_]
            bx0, bx1 = sharding.band_x_range(grid, blo, bhi)
            for j in (a, b):
                x_, y_ = sf.synthetic_uniform(4242 + 1000 * r_ + j, pane_pts, bx0, bx1, BEIJING[2], BEIJING[3])
                xs.append(x_); ys.append(y_)
                obs.append(np.arange(pane_pts, dtype=np.int64) + (r_ * npanes + j) * pane_pts)
        t = time.perf_counter()
        st, eo, ed, ei = O.knn(O.grid(grid_n, *BEIJING), np.concatenate(xs), np.concatenate(ys), np.concatenate(obs),
                               QPOINT[0], QPOINT[1], args.radius, k)
        verified = bool(st == 0 and np.array_equal(eo, o) and np.array_equal(ed, d))
        print(f"oracle check of one window over {world} ranks: {verified} ({time.perf_counter() - t:.1f}s)",
              file=sys.stderr, flush=True)
        assert verified, "all-gathered sliding window differs from the oracle"

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        # the reference evaluates every window from scratch (PointPointKNNQuery.java:158-200):
        # its rate in window points / s on a sample of one window's points, the three lines
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        S = min(args.cpu_sample, pane_pts)
        x, y, obj = host[0]
        xs, ys, os_ = (np.ascontiguousarray(a[:S]) for a in (x, y, obj))
        og = O.grid(grid_n, *BEIJING)
        q5 = (QPOINT[0], QPOINT[1], args.radius, k)

        def final(res):  # (objID, dist) sorted by (dist, objID): the reference's heap in rank order
            st, o, d = res[0], res[1], res[2]
            i = np.lexsort((o, d))
            return st, o[i], d[i]
        cpu = _cpu_lines(args, "window points/s", {
            "mt": (S, lambda T: final(O.knn_mt(og, xs, ys, os_, *q5, T)), f"first {S} points of a window"),
            "single": (S, lambda T: final(O.knn(og, xs, ys, os_, *q5, reference_shaped=True)),
                       f"first {S} points of a window"),
            "omp": (S, lambda T: final(O.knn_mt(og, xs, ys, os_, *q5, T, optimized=True)),
                    f"first {S} points of a window")},
            lambda R: all(R[k_][0] == 0 for k_ in R) and all(
                np.array_equal(R[k_][1], R["mt"][1]) and np.array_equal(R[k_][2], R["mt"][2]) for k_ in R))
    traffic, traffic_src = None, None
    if rank == 0:  # HBM bytes per pane launch from the committed rocprofv3 PMC passes
        import glob

        # newest round first: r<NN>_sliding_pmc.json (tools/pmc_table.py layout) or the older
        # r<NN>_sliding_knn_fused_pmc.json (one kernel, with its points per launch)
        files = glob.glob(os.path.join(ROOT, "profiles", "r*_sliding_pmc.json")) + \
            glob.glob(os.path.join(ROOT, "profiles", "r*_sliding_knn_fused_pmc.json"))
        for f in sorted(files, key=lambda f: (os.path.basename(f).split("_")[0], "knn_fused" not in f), reverse=True):
            with open(f) as fh:
                pm = json.load(fh)
            if "pmc" in pm:
                ent = [v for k_, v in pm["pmc"].items() if "knn_fused_kernel" in k_]
                # the campaign ran the default pane; take it only when it streamed this pane's bytes
                if ent and abs(ent[0]["hbm_read_bytes_corrected"] - 16.0 * pane_pts) < 0.05 * 16.0 * pane_pts:
                    traffic = ent[0]["hbm_read_bytes_corrected"] + ent[0].get("hbm_write_bytes", 0.0)
                    traffic_src = (os.path.relpath(f, ROOT) + ": rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes, "
                                   "median per knn_fused_kernel launch, FETCH_SIZE x2 (gfx950)")
                    break
            elif pm.get("points_per_launch") == pane_pts:
                traffic = pm["traffic_bytes_per_launch"]
                traffic_src = os.path.relpath(f, ROOT) + ": rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE, median per launch"
                break
    if rank == 0:
        avg = scan_ms / 1000.0 / max(scan_n, 1)
        steps = args.steps
        d = {"metric": "points/sec per window (sliding-window kNN k=100)", "value": round(window_pts * steps / elapsed, 1),
             "unit": "window points/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
             "ms_per_step": round(1000.0 * elapsed / steps, 6), "higher_is_better": True,
             "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "f64",
             "data": f"synthetic: java.util.Random-compatible uniform points, Beijing bounds, {npanes} distinct "
                     "device-resident panes cycled",
             "config": {"workload": f"sliding_knn_k{k}_r{args.radius}_{window_pts // 1_000_000}Mpts_grid{grid_n}",
                        "window_points": window_pts, "size_over_slide": W, "pane_points_per_gpu": pane_pts,
                        "k": k, "radius": args.radius, "grid": grid_n, "windows_in_flight": depth,
                        "parallelism": f"cell-column shards x{world}" + (" + RCCL all-gather top-k" if world > 1 else ""),
                        "exchange_batch": B if world > 1 else None, "exchange": xdesc},
             "roofline": {"bound": "hbm", "kernel": "knn_fused (scan of pane i + select of pane i-1)",
                          "achieved": round(16.0 * pane_pts / avg / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(16.0 * pane_pts / avg / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                          "traffic_source": traffic_src,
                          "bytes_per_launch": 16.0 * pane_pts, "avg_launch_us": round(avg * 1e6, 2),
                          "launches_timed": scan_n},
             "scanned_points_per_s": round(pane_pts * world * steps / elapsed, 1),
             "breakdown": {"merge_us": round(1000.0 * merge_ms / max(merge_n, 1), 2),
                           "from_scratch_window_us": round(scratch_us, 2) if scratch_us else None},
             "cpu_baseline": cpu, "verified_vs_whole_window_and_oracle": verified,
             "build": L.gf_build_info().decode()}
        print(json.dumps(d), flush=True)
    L.gf_knn_sliding_destroy(eng)
    if comm is not None:
        comm.destroy()
    if world > 1:
        dist.destroy_process_group()


def _geojson_chunk(args_):
    """Process-pool worker of the GeoJSON multi-core CPU line: the oracle's per-line map."""
    text, = args_
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    x, y, o, t, bl, bk = O.geojson_parse(text, "oID", "timestamp", 1, 480)
    return x, y, bl


def _geojson_pool_baseline(args, text):
    """The GeoJSON map on T processes (Flink map parallelism T): the chunk's lines split into T
    contiguous parts, each parsed by the oracle (Python json per line) in its own process.
    Returns (T, lines/s, sample, results equal the serial oracle)."""
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    T, nproc, model = _host_threads()
    lines_ = text.split(b"\n")[:-1]
    n = len(lines_)
    parts = [b"\n".join(lines_[n * t // T: n * (t + 1) // T]) + b"\n" for t in range(T)]
    with mp.get_context("spawn").Pool(T) as pool:
        pool.map(_geojson_chunk, [(b'{"value":{"type":"Point","coordinates":[1,2]}}\n',)] * T)  # warm workers
        budget = min(args.cpu_seconds / 3.0, 10.0)
        reps, t0 = 0, time.perf_counter()
        while True:
            out = pool.map(_geojson_chunk, [(p_,) for p_ in parts])
            reps += 1
            if time.perf_counter() - t0 >= budget:
                break
        el = time.perf_counter() - t0
    ex, ey, *_ = O.geojson_parse(text, "oID", "timestamp", 1, 480)
    agree = all(o_[2] == -1 for o_ in out) and np.array_equal(np.concatenate([o_[0] for o_ in out]), ex) and \
        np.array_equal(np.concatenate([o_[1] for o_ in out]), ey)
    sample = (f"the {n}-line window x {reps} ({el:.1f}s): oracle geojson_parse (Python json per line) on {T} "
              f"processes, contiguous parts (Flink map parallelism {T}; {nproc} cores, {model})")
    return T, reps * n / el, sample, agree


def bench_csv(args, geojson=False):
    """C1 ingest: 1M-line CSV window (objID, ts, x, y; shortest round-trip doubles, the way Java's
    Double.toString prints them) device-resident as text -> gf_csv_parse (SoA + 100x100 cells),
    then the C1 point-point range query on the parsed window.  value = lines/s of the whole
    text -> range-hits step; the parse kernel's roofline counts text bytes + 40 B/point out.
    geojson: the same with 1M GeoJSON lines (tests/geojson_gen.py: Kafka records and bare
    Features, date-string timestamps in UTC+8) -> gf_geojson_parse (Deserialization.java:149-211)."""
    import torch

    import spatialflink_amd as sf
    from spatialflink_amd import _lib
    from spatialflink_amd.spatialStreams import GfCsvSchema, GfGeojsonSchema, device_text

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from csv_gen import make_csv
    from geojson_gen import lines as geojson_lines

    n = args.points or 1_000_000
    L = _lib.lib()
    host_texts = []
    for j in range(2):
        if geojson:
            host_texts.append((geojson_lines(31 + j, n, 1), None, None, None))
        else:
            host_texts.append(make_csv(n, seed=31 + j)[:4])
    # the GeoJSON oracle is Python (json module per line): its multi-core line runs on a process
    # pool, started before this process touches the GPU (no fork of a GPU-initialised process)
    geo_pool_lines = _geojson_pool_baseline(args, host_texts[(args.steps - 1) % 2][0]) if (
        geojson and not args.no_cpu_baseline) else None
    ctx = _lib.context(0)
    if geojson and args.geojson_locator == "wave":  # (default: one line per lane; older builds lack the flag)
        _lib.check(L.gf_ctx_set_flag(ctx.handle, _lib.FLAG_GEOJSON_WAVE, int(args.geojson_locator == "wave")),
                   ctx.handle, "flag")
    grid = sf.UniformGrid(100, *BEIJING)
    texts = [(t_[0], t_[1], t_[2], t_[3], device_text(t_[0])) for t_ in host_texts]
    nbytes = len(texts[0][0])
    sc = GfGeojsonSchema(b"oID", b"timestamp", 1, 480) if geojson else GfCsvSchema(b",", b"\0\0\0", 0, 1, 2, 3)
    dict_h = sf.ObjIdDict.default(0).handle
    x = torch.empty(n, dtype=torch.float64, device="cuda"); y = torch.empty_like(x)
    o = torch.empty(n, dtype=torch.int64, device="cuda"); ts = torch.empty_like(o)
    cx = torch.empty(n, dtype=torch.int32, device="cuda"); cy = torch.empty_like(cx)
    nout, bl, bk = C.c_int64(), C.c_int64(), C.c_int32()
    qx = np.array([QPOINT[0]]); qy = np.array([QPOINT[1]])
    h = C.c_void_p()
    _lib.check(L.gf_range_pp_plan_create(ctx.handle, C.byref(grid.c_grid), qx.ctypes.data, qy.ctypes.data, 1,
                                         args.radius, 0, 0, C.byref(h)), ctx.handle, "plan")
    words = (n + 63) // 64
    bitmap = torch.empty(words, dtype=torch.int64, device="cuda")
    counts = torch.zeros(2, dtype=torch.int64, device="cuda")
    pts = sf.PointWindow(x, y, o, ts).c_struct()

    def parse(i):
        t = texts[i % 2][4]
        fn = L.gf_geojson_parse if geojson else L.gf_csv_parse_dict
        _lib.check(fn(ctx.handle, dict_h, C.c_void_p(t.data_ptr()), t.numel(), C.byref(sc), C.byref(grid.c_grid),
                      x.data_ptr(), y.data_ptr(), o.data_ptr(), ts.data_ptr(), cx.data_ptr(), cy.data_ptr(),
                      n, C.byref(nout), C.byref(bl), C.byref(bk)), ctx.handle, "parse")

    def step(i):
        parse(i)
        _lib.check(L.gf_range_run(h, C.byref(pts), bitmap.data_ptr(), None, counts.data_ptr()), ctx.handle, "range")

    # the context's FIRST call (no mean line length yet: the staging is sized from the format's
    # default -- ADVICE r05), timed on its own
    torch.cuda.synchronize()
    tcold = time.perf_counter()
    parse(0)
    torch.cuda.synchronize()
    cold_ms = 1000.0 * (time.perf_counter() - tcold)
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    ctx.set_timing((1 << _lib.K_CSV_PARSE) | (1 << _lib.K_RANGE_SCAN))
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    pms, pcnt = ctx.timing(_lib.K_CSV_PARSE)
    rms, rcnt = ctx.timing(_lib.K_RANGE_SCAN)
    ctx.set_timing(0)
    # ingest alone
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(args.steps):
        parse(i)
    torch.cuda.synchronize()
    ingest_s = (time.perf_counter() - t1) / args.steps
    # parity: the last parsed window (texts[(steps-1) % 2]) bit-exact vs the oracle, and its range hits
    j = (args.steps - 1) % 2
    parse(j)
    text = texts[j][0]
    oracle_parse = (lambda t_: O.geojson_parse(t_, "oID", "timestamp", 1, 480)) if geojson else (
        lambda t_: O.csv_parse(t_, ",", [0, 1, 2, 3]))
    ex, ey, eo, et, ebl, ebk = oracle_parse(text)
    # objIDs: the keys decode to the oracle's Strings exactly (numeric Strings are their own key)
    verified = bool(ebl == -1 and np.array_equal(x.cpu().numpy().view(np.int64), ex.view(np.int64))
                    and np.array_equal(y.cpu().numpy().view(np.int64), ey.view(np.int64))
                    and [None if k_ == _lib.OBJID_NULL else b_ for k_, b_ in
                         zip(o.cpu().numpy().tolist(), sf.ObjIdDict.default(0).decode_bytes(o.cpu().numpy()))] == eo
                    and np.array_equal(ts.cpu().numpy(), et))
    og = O.grid(100, *BEIJING)
    ecx, ecy = O.assign_cells(og, ex, ey)
    verified &= bool(np.array_equal(cx.cpu().numpy(), ecx) and np.array_equal(cy.cpu().numpy(), ecy))
    _lib.check(L.gf_range_run(h, C.byref(pts), bitmap.data_ptr(), None, counts.data_ptr()), ctx.handle, "range")
    got = sf.spatialOperators.bitmap_indices(ctx, bitmap, n).astype(np.int64)
    verified &= bool(np.array_equal(got, O.range_pp(og, ex, ey, [QPOINT[0]], [QPOINT[1]], args.radius)))
    L.gf_range_plan_destroy(h)
    cpu = None
    if not args.no_cpu_baseline and geojson:  # the oracle's restatement of the map, Python json per line
        reps, tc = 0, time.perf_counter()
        while True:
            oracle_parse(text)
            reps += 1
            if time.perf_counter() - tc >= min(args.cpu_seconds / 3.0, 10.0):
                break
        ct = time.perf_counter() - tc
        T, rate_mt, samp_mt, agree_mt = geo_pool_lines
        cpu = {"value": round(rate_mt, 1), "unit": "lines/s", "cores": T, "kind": "port",
               "sample": samp_mt, "results_equal_gpu": bool(agree_mt and verified),
               "single_thread": {"value": round(reps * n / ct, 1), "unit": "lines/s", "cores": 1, "kind": "port",
                                 "sample": f"the {n}-line window x {reps} ({ct:.1f}s): oracle geojson_parse (Python "
                                           "json module per line + the map's geometry / property logic), 1 thread"}}
    elif not args.no_cpu_baseline:  # CSV: orc_csv_parse per line (the reference's map restated in C)
        def xy(res):
            return res[0], res[1]
        cpu = _cpu_lines(args, "lines/s", {
            "mt": (n, lambda T: xy(O.csv_parse_mt(text, ",", [0, 1, 2, 3], T)),
                   f"the {n}-line window: orc_csv_parse on contiguous parts (Flink map parallelism)"),
            "single": (n, lambda T: xy(O.csv_parse(text, ",", [0, 1, 2, 3])),
                       f"the {n}-line window: orc_csv_parse (quote removal, Java split rule, Long.valueOf, strtod)")},
            lambda R: all(np.array_equal(R[k_][0], ex) and np.array_equal(R[k_][1], ey) for k_ in R))
    avg_parse = pms / 1000.0 / max(pcnt, 1)
    _line(("GeoJSON" if geojson else "CSV") + " ingest + point-point range", n * args.steps / elapsed, "lines/s",
          args.steps, args.warmup, elapsed,
          ("geojson_wave_kernel" if args.geojson_locator == "wave" else "csv_parse_kernel (GeoJSON lines)")
          if geojson else "csv_parse_kernel",
          float(nbytes + 40 * n), avg_parse,
          {"config": {"workload": f"{'geojson' if geojson else 'csv'}_{n // 1_000_000}Mlines_range_r{args.radius}_grid100",
                      "lines": n,
                      "text_bytes": nbytes, "radius": args.radius},
           "breakdown": {"parse_kernel_us": round(avg_parse * 1e6, 2),
                         "range_kernel_us": round(rms * 1000.0 / max(rcnt, 1), 2),
                         "ingest_call_us": round(ingest_s * 1e6, 2),
                         "ingest_lines_per_s": round(n / ingest_s, 1),
                         "ingest_text_GBps": round(nbytes / ingest_s / 1e9, 2),
                         "cold_first_call_ms": round(cold_ms, 3)},
           **({"geojson_locator": args.geojson_locator} if geojson else {}),
           "cpu_baseline": cpu, "verified_vs_oracle": verified})


def bench_polyknn(args):
    """Polygon-query kNN (PointPolygonKNNQuery.java:245-317, §8f row 4): k = 50, r = 0.5, a
    0.02-degree square around the README query point, 500 x 500 grid, 10M points per window,
    continuous query over a ring of distinct windows (threshold hint carried), depth 2;
    --poly-streams S: consecutive windows alternate over S plans on their own contexts (HIP
    streams), so one window's launches ramp up under the other's tail (each plan carries the
    hint of every S-th window)."""
    import torch

    import spatialflink_amd as sf
    from spatialflink_amd import _lib

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    n = args.points or 10_000_000
    L = _lib.lib()
    grid = sf.UniformGrid(500, *BEIJING)
    h = 0.01
    ring = [(QPOINT[0] - h, QPOINT[1] - h), (QPOINT[0] + h, QPOINT[1] - h), (QPOINT[0] + h, QPOINT[1] + h),
            (QPOINT[0] - h, QPOINT[1] + h), (QPOINT[0] - h, QPOINT[1] - h)]
    P = sf.Polygon([ring], grid)
    wins = _windows(sf, n, 4, 61)
    op = sf.PointPolygonKNNQuery(sf.QueryConfiguration(sf.QueryType.WindowBased), grid)
    ctx, plan = op.plan(0, P, args.radius, args.k)
    # depth 2: window i's select rides in block 0 of window i+1's prefilter scan; depth 3 (the
    # default): in window i+2's, consecutive windows on the plan's two streams -- ONE plan, the
    # product path a Flink shim holding one PointPolygonKNNQuery plan gets
    depth = args.pipeline
    _lib.check(L.gf_knn_plan_set_pipeline(plan, depth), ctx.handle, "pipeline")
    ctxs, plans = [ctx], [plan]
    cs = sf.PolygonSet([P]).c_struct()
    for _ in range(max(1, args.poly_streams) - 1):
        c2 = _lib.Context(0)
        h2 = C.c_void_p()
        _lib.check(L.gf_knn_ppoly_plan_create(c2.handle, C.byref(grid.c_grid), C.byref(cs), float(args.radius),
                                              int(args.k), 0, 0, C.byref(h2)), c2.handle, "plan")
        _lib.check(L.gf_knn_plan_set_pipeline(h2, depth), c2.handle, "pipeline")
        ctxs.append(c2)
        plans.append(h2)
    nst = len(plans)
    recs = sf.PinnedRecords(args.warmup + args.steps, args.k)
    pts = [w[2].c_struct() for w in wins]

    def step(i):
        _lib.check(L.gf_knn_enqueue(plans[i % nst], C.byref(pts[i % 4]), C.c_void_p(recs.ptr(i))),
                   ctxs[i % nst].handle, "enqueue")

    def flush_all():
        for c, pl in zip(ctxs, plans):
            _lib.check(L.gf_knn_plan_flush(pl), c.handle, "flush")
        for c in ctxs:
            c.synchronize()
        torch.cuda.synchronize()

    for i in range(args.warmup):
        step(i)
    flush_all()
    for c in ctxs:
        c.set_timing((1 << _lib.K_KNN_SCAN) | (1 << _lib.K_KNN_SAMPLE) | (1 << _lib.K_KNN_SELECT))
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i)
    flush_all()
    elapsed = time.perf_counter() - t0
    sms = scnt = pms = pcnt = lms = lcnt = 0
    for c in ctxs:
        a_ms, a_n = c.timing(_lib.K_KNN_SCAN)
        b_ms, b_n = c.timing(_lib.K_KNN_SAMPLE)
        c_ms, c_n = c.timing(_lib.K_KNN_SELECT)
        sms, scnt, pms, pcnt, lms, lcnt = sms + a_ms, scnt + a_n, pms + b_ms, pcnt + b_n, lms + c_ms, lcnt + c_n
        c.set_timing(0)
    for pl in plans[1:]:
        L.gf_knn_plan_destroy(pl)
    fallbacks = sum(1 for i in range(args.warmup, args.warmup + args.steps) if recs.decode(i)[0] != 0)
    verified, cpu = None, None
    if not args.no_verify:  # the first window against the oracle
        x, y, w = wins[args.warmup % 4]
        st, o, d, ix = recs.decode(args.warmup)
        og, oP, oid = O.grid(500, *BEIJING), O.Polygons([P.rings]), np.arange(n, dtype=np.int64)
        m, eo, ed, ei = O.knn_ppoly_mt(og, x, y, oid, oP, args.radius, args.k, _host_threads()[0])
        verified = bool(st == 0 and np.array_equal(o, eo) and np.array_equal(d, ed) and np.array_equal(ix, ei))
        if not args.no_cpu_baseline:
            def same(res):
                return all(r[0] == m and all(np.array_equal(a, b) for a, b in zip(r[1:], (eo, ed, ei)))
                           for r in res.values())
            cpu = _cpu_lines(args, "points/s", {
                "mt": (n, lambda T: O.knn_ppoly_mt(og, x, y, oid, oP, args.radius, args.k, T),
                       f"the whole {n}-point window: PointPolygonKNNQuery restated (polygon G/C cell filter, "
                       "JTS point-polygon distance, objID dedupe, first k) over point parts"),
                "single": (n, lambda T: O.knn_ppoly(og, x, y, oid, oP, args.radius, args.k),
                           f"the whole {n}-point window"),
            }, same)
    avg = sms / 1000.0 / max(scnt, 1)
    # windows in flight: a launch's own duration counts shared time several times, so the rate
    # is bytes per window over the window interval (as the range lines)
    interval = nst > 1 or depth >= 3
    basis = (f"bytes per window / window interval ({nst} plan(s), depth {depth}: launches of consecutive windows "
             "overlap; includes host work)" if interval else "bytes per window / average prefilter-scan launch")
    kern = {1: "knn_poly_scan", 2: "knn_poly_fused (prefilter scan + the previous window's select in block 0)",
            3: "knn_poly_fused (prefilter scan + the select of the window two back in block 0; consecutive "
               "windows on the plan's two streams)",
            4: "knn_poly_fused (prefilter scan + the select of the window three back in block 0; consecutive "
               "windows on the plan's three streams)"}[depth]
    _line("polygon-query kNN k=%d" % args.k, n * args.steps / elapsed, "points/s", args.steps, args.warmup, elapsed,
          kern, 16.0 * n, elapsed / args.steps if interval else avg,
          {"config": {"workload": f"knn_ppoly_k{args.k}_r{args.radius}_{n // 1_000_000}Mpts_grid500_square0.02",
                      "points_per_window": n, "k": args.k, "radius": args.radius, "pipeline_depth": depth,
                      "plans": nst, "windows_in_flight": nst * (depth - 1 if depth >= 3 else 1)},
           "breakdown": {"scan_us": round(avg * 1e6, 2), "sample_us": round(1000 * pms / max(pcnt, 1), 2),
                         "select_us": round(1000 * lms / max(lcnt, 1), 2), "achieved_basis": basis},
           "fallback_windows": fallbacks, "verified_vs_oracle": verified,
           **({"cpu_baseline": cpu} if cpu else {})})


def bench_bucket(args):
    """K2 bucketing by cell (north-star subsystem 2, the keyBy(gridID) shuffle,
    PointPointRangeQuery.java:144-148): gf_bucket_by_cell over 10M-point windows of the C2 grid
    (500 x 500).  A step = one window: the stable radix passes + bucket offsets.  Algorithmic
    bytes: x, y in (16 B/point) + the permutation out (4 B/point) + cell_start (4 B/bucket); the
    passes move 28 B/point more (keys, indices) -- the roofline counts only the former."""
    import torch

    import spatialflink_amd as sf
    from spatialflink_amd import _lib

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    n = args.points or 10_000_000
    grid_n = args.grid
    L = _lib.lib()
    grid = sf.UniformGrid(grid_n, *BEIJING)
    nwin = 4
    wins = _windows(sf, n, nwin, 91)
    ctx = _lib.context(0)
    perm = torch.empty(n, dtype=torch.int32, device="cuda")
    start = torch.empty(grid_n * grid_n + 2, dtype=torch.int32, device="cuda")
    pts = [w[2].c_struct() for w in wins]

    def step(i):
        _lib.check(L.gf_bucket_by_cell(ctx.handle, C.byref(grid.c_grid), C.byref(pts[i % nwin]), perm.data_ptr(),
                                       start.data_ptr()), ctx.handle, "gf_bucket_by_cell")

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the per-kernel breakdown from a second pass of the same steps with HIP events around every
    # launch (outside the timed region: the event records add host work between the launches)
    ctx.set_timing(1 << _lib.K_BUCKET)
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    ms, cnt = ctx.timing(_lib.K_BUCKET)
    ctx.set_timing(0)
    verified = None
    if not args.no_verify:  # the exact permutation (stable: arrival order inside a bucket)
        step(0)
        x, y, _ = wins[0]
        og = O.grid(grid_n, *BEIJING)
        cx, cy = O.assign_cells(og, x, y)
        valid = (cx >= 0) & (cy >= 0) & (cx < grid_n) & (cy < grid_n)
        key = np.where(valid, cy.astype(np.int64) * grid_n + cx, grid_n * grid_n)
        ep = np.argsort(key, kind="stable")
        verified = bool(np.array_equal(perm.cpu().numpy().view(np.uint32).astype(np.int64), ep))
    per_window = elapsed / args.steps
    bytes_alg = 20.0 * n + 4.0 * (grid_n * grid_n + 2)
    _line("K2 bucketing by cell", n * args.steps / elapsed, "points/s", args.steps, args.warmup, elapsed,
          "radix hist + scatter passes (gf_bucket_by_cell)", bytes_alg, per_window,
          {"config": {"workload": f"bucket_by_cell_{n // 1_000_000}Mpts_grid{grid_n}", "points_per_window": n,
                      "grid": grid_n},
           "breakdown": {"kernel_us_per_window": round(1000.0 * ms / max(args.steps, 1), 2),
                         "launches_per_window": cnt / args.steps,
                         "breakdown_basis": "a second pass of the same steps with HIP events per launch",
                         "achieved_basis": "algorithmic bytes / whole call (all passes + scans)"},
           "verified_vs_oracle": verified})


def run(args):
    if args.workload in ("range", "ppoly"):
        bench_range(args, polygons=args.workload == "ppoly")
    elif args.workload == "join":
        bench_join(args)
    elif args.workload == "pjoin":
        bench_pjoin(args)
    elif args.workload == "sliding":
        bench_sliding(args)
    elif args.workload == "csv":
        bench_csv(args)
    elif args.workload == "geojson":
        bench_csv(args, geojson=True)
    elif args.workload == "polyknn":
        bench_polyknn(args)
    elif args.workload == "bucket":
        bench_bucket(args)
    else:
        raise SystemExit(f"unknown workload {args.workload}")
