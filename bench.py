#!/usr/bin/env python3
"""bench.py -- window-evaluation throughput of the GeoFlink kNN hot path on MI355X.

Workload (BASELINE.json configs[1]): continuous kNN, k = 50, radius 0.5 around the README
query point (116.414899, 39.920374), 500 x 500 UniformGrid over Beijing bounds, 10M points
per window per GPU, synthetic java.util.Random-compatible uniform points.  A step = one
window evaluated end to end on the device (sample -> scan -> select, plus the RCCL top-k
all-gather + merge when N > 1); the final kernel writes the result record straight into mapped
pinned host memory (PinnedRecords), so no copy kernel runs per window.
Windows are device-resident when the timed region starts.

N > 1 (one process per GPU, torchrun): the window is sharded by grid-cell column bands, each
rank holds 10M points of its band (weak scaling), per-rank top-k records are all-gathered over
RCCL and merged on every rank.

Prints ONE JSON line (rank 0) with the metric, a roofline object for the dominant kernel
(knn_scan, HIP events on its stream over the timed region) and the CPU baselines (the oracle's
reference-shaped evaluator on every thread of the CPU share and on one, plus an optimised OpenMP
scan; see cpu_baselines).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BEIJING = (115.5, 117.6, 39.6, 41.1)
QPOINT = (116.414899, 39.920374)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "points/sec per window (kNN k=50, range r) at 1/2/4/8 MI355X; % HBM roofline"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _timed_reps(fn, budget_s):
    reps, t = 0, time.perf_counter()
    while True:
        out = fn()
        reps += 1
        if time.perf_counter() - t >= budget_s:
            return reps, time.perf_counter() - t, out


def cpu_baselines(args, O, og, window, gpu_result, n):
    """SURVEY.md 8(d) CPU baselines on this host, in the same run (rank 0, N = 1), each a
    C restatement (the JVM/Flink operator cannot run here):
      value           the reference-shaped operator on every thread of this process's CPU share,
                      shaped as Flink runs it with that parallelism (conf/geoflink-conf.yml:55;
                      keyBy(gridID) over subtasks, PointPointRangeQuery.java:144-148): string cell
                      IDs, HashSet C/G filter, hash shuffle, per-cell PriorityQueue, windowAll merge;
      single_thread   the same evaluator on one thread (a bounded sample);
      optimized_scan  an optimised OpenMP C scan (integer cell test, distance prefilter against
                      the running k-th distance, per-thread top-k-distinct heaps) -- the honest
                      best-effort CPU line.
    Every line's result is checked against the GPU's record of the same window."""
    x, y, obj = window
    nproc, model = O.host_cpu()
    threads = min(nproc, int(os.environ.get("OMP_NUM_THREADS") or nproc))
    budget = max(1.0, args.cpu_seconds / 3.0)
    q = (QPOINT[0], QPOINT[1], args.radius, args.k)
    reps, t, res = _timed_reps(lambda: O.knn_mt(og, x, y, obj, *q, threads), budget)
    go, gd, gi = gpu_result
    # the reference's result is its PriorityQueue in heap order: compare as (d, objID)-sorted
    o_ = np.lexsort((res[1], res[2])) if res[0] == 0 else None
    agree = bool(res[0] == 0 and np.array_equal(res[1][o_], go) and np.array_equal(res[2][o_], gd))
    S = min(args.cpu_sample, n)
    xs, ys, os_ = (np.ascontiguousarray(a[:S]) for a in (x, y, obj))
    reps1, t1, _ = _timed_reps(lambda: O.knn(og, xs, ys, os_, *q, reference_shaped=True), budget)
    repso, to, reso = _timed_reps(lambda: O.knn_mt(og, x, y, obj, *q, threads, optimized=True), budget)
    agree_o = bool(reso[0] == 0 and np.array_equal(reso[1], go) and np.array_equal(reso[2], gd)
                   and np.array_equal(reso[3], gi))
    log(f"CPU baselines ({threads} threads of {nproc}, {model}): reference-shaped {reps * n / t:.3g} pts/s, "
        f"1 thread {reps1 * S / t1:.3g}, optimised scan {repso * n / to:.3g}")
    return {"value": round(reps * n / t, 1), "unit": "points/s", "cores": threads, "kind": "port",
            "nproc": nproc, "cpu_model": model,
            "threads_note": "threads = this process's CPU share on the GPU box (OMP_NUM_THREADS), of nproc",
            "sample": (f"the whole {n}-point window x {reps} ({t:.1f}s): oracle's reference-shaped operator on "
                       f"{threads} threads shaped as Flink's keyBy(gridID) parallelism (source subtasks: string cell "
                       "IDs + HashSet C/G filter + JTS distance; hash shuffle; key subtasks: per-cell "
                       "PriorityQueue; one windowAll merge), C restatement of the Java operator"),
            "result_equals_gpu": agree,
            "single_thread": {"value": round(reps1 * S / t1, 1), "unit": "points/s", "cores": 1, "kind": "port",
                              "sample": f"first {S} points of the window x {reps1} ({t1:.1f}s), same evaluator"},
            "optimized_scan": {"value": round(repso * n / to, 1), "unit": "points/s", "cores": threads,
                               "kind": "port", "result_equals_gpu": agree_o,
                               "sample": (f"the whole {n}-point window x {repso} ({to:.1f}s): optimised OpenMP C "
                                          "scan (oracle/cpu_scan.c: integer Chebyshev cell test, squared-distance "
                                          "prefilter against each thread's k-th distance, per-thread "
                                          "top-k-distinct heap, one merge)")}}


def intern_fixed(sdict, prefix: bytes, values, digits: int):
    """Intern the Strings prefix + "%0{digits}d" % v of int64 values into `sdict` (gf_objid_intern on
    one fixed-width blob) -> int64 keys."""
    v = np.asarray(values, np.int64)
    w = len(prefix) + digits
    a = np.empty((len(v), w), np.uint8)
    a[:, :len(prefix)] = np.frombuffer(prefix, np.uint8)
    for j in range(digits):
        a[:, len(prefix) + j] = 48 + (v // 10 ** (digits - 1 - j)) % 10
    offs = np.arange(len(v) + 1, dtype=np.int64) * w
    keys = np.empty(len(v), np.int64)
    from spatialflink_amd import _lib

    _lib.check(_lib.lib().gf_objid_intern(sdict.handle, a.tobytes(), offs.ctypes.data, len(v), keys.ctypes.data),
               sdict.ctx.handle, "gf_objid_intern")
    return keys


class PinnedStringRecords:
    """A ring of string records (sharding.string_record_bytes) in mapped pinned host memory."""

    def __init__(self, count: int, k: int, cap: int):
        from spatialflink_amd import _lib, sharding

        self.k, self.cap, self.count = int(k), int(cap), int(count)
        self.bytes = sharding.string_record_bytes(k, cap)
        p = ctypes.c_void_p()
        _lib.check(_lib.lib().gf_pinned_alloc(self.bytes * self.count, ctypes.byref(p)), None, "gf_pinned_alloc")
        self._base = p.value
        self.view = np.ctypeslib.as_array((ctypes.c_uint8 * (self.bytes * self.count)).from_address(self._base))

    def ptr(self, i: int) -> int:
        return self._base + (i % self.count) * self.bytes

    def decode(self, i: int):
        """-> (status, objID ints parsed from "veh%09d", dist, idx)"""
        from spatialflink_amd import sharding

        j = i % self.count
        st, strs, d, ix = sharding.decode_string_record(self.view[j * self.bytes:(j + 1) * self.bytes].tobytes(),
                                                         self.k, self.cap)
        return st, np.array([int(s_[3:]) for s_ in strs], np.int64), d, ix


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch_ranks(args):
    """`--gpus N` is the job's parallelism (env.setParallelism, StreamingJob.java:177): one process
    per GPU.  Launched by hand (no WORLD_SIZE in the environment) with N > 1, this process starts
    `python -m torch.distributed.run --nproc-per-node N bench.py <same args>` as a CHILD -- before
    anything here has touched the GPU (no torch import yet) -- relays its output (rank 0 prints the
    one JSON line) and returns its exit code.  Under a launcher, WORLD_SIZE must equal N.
    -> None when this process is a rank (or N == 1), else the launcher's exit code."""
    import subprocess

    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (the launcher started a different "
                "number of ranks)")
            return 2
        return None
    if args.gpus < 1:
        log("bench.py: --gpus must be >= 1")
        return 2
    if args.gpus == 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"bench.py: launching {args.gpus} ranks: {' '.join(cmd)}")
    sys.stdout.flush()
    return subprocess.run(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1")).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--points", type=int, default=None, help="points per window per GPU (kNN default 10M)")
    ap.add_argument("--workload", default="knn", choices=("knn", "range", "ppoly", "join", "pjoin", "sliding", "csv", "geojson", "polyknn", "bucket"),
                    help="knn = the headline line (BASELINE configs[1]); range/ppoly/join/pjoin/sliding/csv/polyknn/"
                         "bucket: tools/bench_workloads.py")
    ap.add_argument("--range-blocks", default="0", help="range/ppoly scan blocks, comma list = sweep (0 = auto)")
    ap.add_argument("--range-defer", default="0", help="range/ppoly candidate tests: 0 auto, 1 inline, 2 deferred (list = sweep)")
    ap.add_argument("--range-streams", type=int, default=3,
                    help="range/ppoly: consecutive windows alternate over this many contexts (HIP streams)")
    ap.add_argument("--range-batch", type=int, default=0,
                    help="range/ppoly: windows per gf_range_run_batch launch (0 = auto: 16 for windows of <= 2M "
                         "points, else 1 = one gf_range_run per window)")
    ap.add_argument("--no-indices", action="store_true",
                    help="range/ppoly: leave the index list out of the step (bitmap + counts only; ablation)")
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--radius", type=float, default=0.5)
    ap.add_argument("--grid", type=int, default=500)
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU baseline budget, split over its three lines (rank 0, N=1)")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--join-stream", action="store_true",
                    help="join workload: experiment -- bucket only the query side, stream the ordinary points")
    ap.add_argument("--poly-streams", type=int, default=1,
                    help="polyknn: consecutive windows alternate over this many plans / contexts (default 1: one "
                         "plan, its depth-3 pipeline keeps two windows in flight)")
    ap.add_argument("--join-streams", type=int, default=2,
                    help="join workload: windows in flight (consecutive windows alternate over this many contexts)")
    ap.add_argument("--join-sync", action="store_true",
                    help="join workload: gf_join_pp per window (pair count read back) instead of gf_join_pp_async")
    ap.add_argument("--clustered", action="store_true",
                    help="BASELINE.md section 3 clustered variant: 80%% of the points in 8 Gaussian hot spots (sigma 0.01)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--geojson-locator", default="lane", choices=("lane", "wave"),
                    help="geojson: members located by the wave-per-line scan or the r05 one-lane-per-line locator")
    ap.add_argument("--windows", type=int, default=4, help="distinct resident windows cycled through")
    ap.add_argument("--timing-period", type=int, default=5,
                    help="HIP events around every N-th launch of the timed kernel (fewer events, less overhead)")
    ap.add_argument("--exchange-batch", type=int, default=8,
                    help="N > 1: windows whose top-k records share one RCCL all-gather + one merge launch")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo: rehearse the N > 1 path with several ranks on one GPU (not a benchmark)")
    ap.add_argument("--exchange", default="auto", choices=("auto", "rccl", "torch"),
                    help="N > 1 kNN record exchange: rccl = the C ABI's communicator (gf_knn_exchange_batch, "
                         "the Java drop-in's path); torch = torch.distributed all-gather; auto = rccl on nccl")
    ap.add_argument("--scan-blocks", type=int, default=0, help="kNN scan grid (0 = auto: 4 blocks per CU)")
    ap.add_argument("--string-objids", action="store_true",
                    help="objIDs are dictionary Strings (\"veh%%09d\", MN_Q1.java:52's deviceId): N > 1 exchanges "
                         "string records (gf_knn_attach_strings + gf_knn_merge_dev_strings)")
    ap.add_argument("--pipeline", type=int, default=None, choices=(1, 2, 3, 4),
                    help="windows in flight: 2 overlaps window i's select with window i+1's scan; 3 also "
                         "overlaps consecutive windows' launches on two streams, 4 on three (default: 3 "
                         "for point kNN -- depth 4 measured 28.5 vs 24.6 us -- and 4 for polygon kNN, "
                         "30.3 vs 33.8 us)")
    args = ap.parse_args()
    launched = _launch_ranks(args)
    if launched is not None:
        sys.exit(launched)
    if args.pipeline is None:
        args.pipeline = 4 if args.workload == "polyknn" else 3
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_workloads as W

    W.CLUSTERED = args.clustered
    if args.workload != "knn":
        W.run(args)
        return
    if args.points is None:
        args.points = 10_000_000

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
    dev = torch.device("cuda", torch.cuda.current_device())

    import spatialflink_amd as sf
    from spatialflink_amd import _lib, sharding
    from spatialflink_amd.spatialOperators import knn_record_bytes

    # ---------------- data: this rank's shard of the window ----------------
    grid = sf.UniformGrid(args.grid, *BEIJING)
    n = args.points
    if world == 1:
        xlo, xhi = BEIJING[0], BEIJING[1]
    else:
        lo, hi = sharding.column_bands(args.grid, world)[rank]
        xlo, xhi = sharding.band_x_range(grid, lo, hi)
    # a ring of distinct windows: consecutive steps never evaluate the same data (the kNN
    # threshold hint carried from window to window is validated on fresh points every step)
    t = time.perf_counter()
    wins, host_windows = [], []
    for j in range(args.windows):
        x, y = W.gen_points(sf, 42 + 1000 * rank + j, n, xlo, xhi)
        obj = np.arange(rank * n, (rank + 1) * n, dtype=np.int64)
        wins.append(sf.PointWindow.from_numpy(x, y, obj, device=dev.index))
        host_windows.append((x, y, obj))
    torch.cuda.synchronize()
    log(f"[rank {rank}] {args.windows} window shards x {n} points, x in [{xlo}, {xhi}): "
        f"generated+uploaded in {time.perf_counter()-t:.2f}s")
    sdict, scap = None, 0
    if args.string_objids:
        # every window of this rank carries the objIDs rank*n .. as the Strings "veh%09d", interned
        # into this rank's own dictionary (ids assigned in this rank's first-occurrence order, so
        # another rank's keys for the same String differ); "veh%09d" orders like its number, so the
        # oracle on the integers is the String contract
        t = time.perf_counter()
        sdict = sf.ObjIdDict(dev.index)
        keys = intern_fixed(sdict, b"veh", np.arange(rank * n, (rank + 1) * n, dtype=np.int64), 9)
        kt = torch.from_numpy(keys).to(dev)
        wins = [sf.PointWindow(w_.x, w_.y, kt, w_.timeStampMillisec) for w_ in wins]
        scap = 16 * args.k + 64
        log(f"[rank {rank}] {n} String objIDs interned in {time.perf_counter()-t:.2f}s")
    w = wins[0]

    conf = sf.QueryConfiguration(sf.QueryType.WindowBased)
    q = sf.Point("q", QPOINT[0], QPOINT[1], 0, grid)
    op = sf.PointPointKNNQuery(conf, grid)
    ctx, plan = op.plan(dev.index, q, args.radius, args.k)
    _lib.check(_lib.lib().gf_knn_plan_set_index_base(plan, rank * n), ctx.handle, "index base")
    _lib.check(_lib.lib().gf_knn_plan_set_pipeline(plan, args.pipeline), ctx.handle, "pipeline")
    if args.scan_blocks:
        _lib.check(_lib.lib().gf_knn_plan_set_tuning(plan, args.scan_blocks, 1, 1), ctx.handle, "tuning")
    lag = args.pipeline - 1  # depth d: window i's record is written by enqueue i+d-1 (or the flush)
    rb = knn_record_bytes(args.k)
    B = max(1, args.exchange_batch)
    slots = torch.zeros(2, B, rb, dtype=torch.uint8, device=dev)  # two groups of B device records
    total_steps = args.warmup + args.steps
    host = sf.PinnedRecords(total_steps, args.k)
    hstr = PinnedStringRecords(total_steps, args.k, scap) if (sdict is not None and world > 1) else None
    L = _lib.lib()
    pts = [w_.c_struct() for w_ in wins]
    pts_ref = [ctypes.byref(p_) for p_ in pts]
    enqueue = L.gf_knn_enqueue

    pending = [0]  # first window whose record has not been exchanged yet
    # Numeric objIDs: a group's exchange (RCCL all-gather + merge) runs on a SIDE stream with a
    # context of its own, so the next group's windows keep streaming while it is in flight (the
    # slots are double-buffered); the first window of group g + 2 waits for group g's exchange
    # (done long before: a group is B windows of work).  String records stay on the plan's stream.
    comm, xdesc = sharding.open_comm(dev.index, args.dist_backend, args.exchange) if world > 1 else (None, None)
    if world > 1:
        log(f"[rank {rank}] record exchange: {xdesc}")
    side = torch.cuda.Stream(dev) if (world > 1 and hstr is None) else None
    xctx = None
    if side is not None:
        xctx = _lib.Context(dev.index)
        xctx.set_stream(side.cuda_stream)
    slot_free = [None, None]  # per slot parity: event after the exchange that last read it

    def exchange(first, lo, hi):  # windows [lo, hi] of one group: one all-gather + one merge launch
        g = (lo - first) // B
        if hstr is not None:  # String objIDs: the records travel with their Strings, merged by String
            if comm is not None:
                comm.exchange_strings_batch(slots[g % 2, : hi - lo + 1], args.k, scap, sdict, hstr.ptr(lo))
            else:
                sharding.allgather_knn_records_strings(slots[g % 2, : hi - lo + 1], args.k, scap, sdict, hstr.ptr(lo))
            if args.pipeline >= 3:
                # depth >= 3 writes windows' records on the plan's other streams: they must not
                # reuse slots[g % 2] (group g + 2) before this all-gather + merge have read them
                _lib.check(L.gf_ctx_fork(ctx.handle), ctx.handle, "gf_ctx_fork")
        else:
            side.wait_stream(torch.cuda.current_stream(dev))  # the group's records are complete
            with torch.cuda.stream(side):
                if comm is not None:
                    comm.exchange_batch(slots[g % 2, : hi - lo + 1], args.k, host.ptr(lo), ctx=xctx)
                else:
                    sharding.allgather_knn_records_batch(slots[g % 2, : hi - lo + 1], args.k, host.ptr(lo), ctx=xctx)
                ev = torch.cuda.Event()
                ev.record(side)
            slot_free[g % 2] = ev
        pending[0] = hi + 1

    def step(i, first):
        if world == 1:  # the select writes the final record straight into pinned host memory
            st = enqueue(plan, pts_ref[i % args.windows], host.ptr(i))
            if st:
                _lib.check(st, ctx.handle, "gf_knn_enqueue")
        else:
            if i == first:
                pending[0] = first
            g, w_ = divmod(i - first, B)
            if w_ == 0 and slot_free[g % 2] is not None:  # group g - 2's exchange has read these slots
                torch.cuda.current_stream(dev).wait_event(slot_free[g % 2])
                slot_free[g % 2] = None
                if args.pipeline >= 3:  # the plan's other streams write records too
                    _lib.check(L.gf_ctx_fork(ctx.handle), ctx.handle, "gf_ctx_fork")
            _lib.check(enqueue(plan, pts_ref[i % args.windows], slots[g % 2, w_].data_ptr()), ctx.handle, "enqueue")
            c = i - lag  # this window's record is complete now
            if c >= first and (c - first) % B == B - 1:
                if args.pipeline >= 3:  # windows' records are written on the plan's other streams too
                    L.gf_ctx_join(ctx.handle)
                exchange(first, c - B + 1, c)

    def drain(first, last):
        _lib.check(L.gf_knn_plan_flush(plan), ctx.handle, "flush")  # joins the second stream
        while world > 1 and pending[0] <= last:  # the groups still pending (up to lag / B + 1 of them)
            lo = pending[0]
            exchange(first, lo, min(last, first + ((lo - first) // B + 1) * B - 1))

    for i in range(args.warmup):
        step(i, 0)
    drain(0, args.warmup - 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    ctx.set_timing_period(args.timing_period)
    ctx.set_timing(1 << _lib.K_KNN_SCAN)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.warmup, total_steps):
        step(i, args.warmup)
    drain(args.warmup, total_steps - 1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    scan_ms, scan_n = ctx.timing(_lib.K_KNN_SCAN)
    ctx.set_timing(0)
    ctx.set_timing_period(1)
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # ---------------- validate every timed window's record ----------------
    per_window = {}
    fallbacks = 0
    for i in range(args.warmup, total_steps):
        if hstr is not None:
            st, o, d, ix = hstr.decode(i)
        else:
            st, o, d, ix = host.decode(i)
            if sdict is not None and st == 0:  # one rank: the keys of its own dictionary
                o = np.array([int(s_[3:]) for s_ in sdict.decode_bytes(o)], np.int64)
        if st != 0:
            fallbacks += 1
            continue
        j = i % args.windows
        if j in per_window:
            assert np.array_equal(per_window[j][0], o) and np.array_equal(per_window[j][1], d), "non-deterministic"
        else:
            per_window[j] = (o, d, ix)
    assert fallbacks == 0, f"{fallbacks} windows needed the exact fallback inside the timed region"

    # per-kernel breakdown (separate, untimed pass), steady state and cold (no hint: sample each window)
    kid_all = (1 << _lib.K_KNN_SCAN) | (1 << _lib.K_KNN_SAMPLE) | (1 << _lib.K_KNN_SELECT)
    breakdown = {}
    for tag, hint in (("", 1), ("cold_", 0)):
        _lib.check(_lib.lib().gf_knn_plan_set_hint(plan, hint), ctx.handle, "hint")
        # both streams busy before the first timed event (an event recorded on an idle stream
        # can carry the timestamp of that stream's last, long-finished command)
        for i in range(4):
            enqueue(plan, pts_ref[i % args.windows], slots[0, i % B].data_ptr())
        ctx.set_timing(kid_all)
        for i in range(12):
            enqueue(plan, pts_ref[i % args.windows], slots[0, i % B].data_ptr())
        L.gf_knn_plan_flush(plan)
        for name, kid in (("sample", _lib.K_KNN_SAMPLE), ("scan", _lib.K_KNN_SCAN), ("select", _lib.K_KNN_SELECT)):
            ms, cnt = ctx.timing(kid)
            breakdown[tag + name + "_us"] = round(1000.0 * ms / max(cnt, 1), 2)
        ctx.set_timing(0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(20):
            enqueue(plan, pts_ref[i % args.windows], slots[0, i % B].data_ptr())
        L.gf_knn_plan_flush(plan)
        torch.cuda.synchronize()
        breakdown[tag + "window_us"] = round(1e6 * (time.perf_counter() - t) / 20, 2)
    _lib.check(_lib.lib().gf_knn_plan_set_hint(plan, 1), ctx.handle, "hint")

    # host-buffer boundary (never part of `value`): windows handed over in host memory.  kNN
    # reads x, y, objID (24 B/point; ts is never uploaded).  Single-upload times (pinned and
    # pageable), then the host-resident pipeline: NH distinct pinned host windows streamed
    # through two gf_windows -- upload(i+1) on the window's copy stream overlaps evaluate(i)
    pcie = None
    if rank == 0 and world == 1:
        bpp = 24
        NH = 3
        pins, hws = [], []
        for j in range(NH):
            pin = ctypes.c_void_p()
            _lib.check(L.gf_pinned_alloc(bpp * n, ctypes.byref(pin)), None, "pinned")
            pv = np.ctypeslib.as_array((ctypes.c_uint8 * (bpp * n)).from_address(pin.value))
            for c_, a_ in enumerate(host_windows[j % args.windows]):
                pv[8 * n * c_: 8 * n * (c_ + 1)] = a_.view(np.uint8)
            pins.append(pin)
        for _ in range(2):
            hw = ctypes.c_void_p()
            _lib.check(L.gf_window_create(ctx.handle, n, ctypes.byref(hw)), ctx.handle, "window")
            hws.append(hw)
        cols = lambda j: [pins[j].value + 8 * n * c_ for c_ in range(3)] + [None]  # noqa: E731
        res = {}
        x0, y0, o0 = host_windows[0]
        for tag, ptrs in (("pageable", [x0.ctypes.data, y0.ctypes.data, o0.ctypes.data, None]), ("pinned", cols(0))):
            best = 1e9
            for _ in range(3):
                torch.cuda.synchronize()
                t = time.perf_counter()
                _lib.check(L.gf_window_upload(hws[0], *ptrs, n), ctx.handle, "upload")
                gp = _lib.GfPoints()
                _lib.check(L.gf_window_points(hws[0], ctypes.byref(gp)), ctx.handle, "points")
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t)
            res[tag] = best

        def host_pipeline(steps):
            _lib.check(L.gf_window_upload(hws[0], *cols(0), n), ctx.handle, "upload")
            for i in range(steps):
                if i + 1 < steps:  # next window's copy, behind everything enqueued so far
                    _lib.check(L.gf_window_upload(hws[(i + 1) % 2], *cols((i + 1) % NH), n), ctx.handle, "upload")
                gp = _lib.GfPoints()
                _lib.check(L.gf_window_points(hws[i % 2], ctypes.byref(gp)), ctx.handle, "points")
                _lib.check(enqueue(plan, ctypes.byref(gp), slots[0, i % B].data_ptr()), ctx.handle, "enqueue")
            _lib.check(L.gf_knn_plan_flush(plan), ctx.handle, "flush")

        def host_pipeline_mapped(steps):  # 16 B per point: objID read in place from pinned host memory
            _lib.check(L.gf_window_upload_mapped(hws[0], *cols(0)[:3], n), ctx.handle, "upload_mapped")
            for i in range(steps):
                if i + 1 < steps:
                    _lib.check(L.gf_window_upload_mapped(hws[(i + 1) % 2], *cols((i + 1) % NH)[:3], n), ctx.handle,
                               "upload_mapped")
                gp = _lib.GfPoints()
                _lib.check(L.gf_window_points(hws[i % 2], ctypes.byref(gp)), ctx.handle, "points")
                _lib.check(enqueue(plan, ctypes.byref(gp), slots[0, i % B].data_ptr()), ctx.handle, "enqueue")
            _lib.check(L.gf_knn_plan_flush(plan), ctx.handle, "flush")

        hsteps = 12
        host_pipeline_mapped(4)
        torch.cuda.synchronize()
        t = time.perf_counter()
        host_pipeline_mapped(hsteps)
        torch.cuda.synchronize()
        hpipe16 = (time.perf_counter() - t) / hsteps
        for i in range(max(0, hsteps - B), hsteps):  # == the device-resident results of the same windows
            st_, o_, d_, _ = sf.spatialOperators.decode_knn_record(slots[0, i % B].cpu().numpy().tobytes(), args.k)
            ref = per_window.get((i % NH) % args.windows) if (i % NH) < args.windows else None
            if ref is not None and sdict is None:
                assert st_ == 0 and np.array_equal(ref[0], o_) and np.array_equal(ref[1], d_), "mapped-objID mismatch"
        host_pipeline(4)
        torch.cuda.synchronize()
        t = time.perf_counter()
        host_pipeline(hsteps)
        torch.cuda.synchronize()
        hpipe = (time.perf_counter() - t) / hsteps
        # the pipeline's last records == the device-resident results of the same windows
        for i in range(max(0, hsteps - B), hsteps):
            st_, o_, d_, _ = sf.spatialOperators.decode_knn_record(slots[0, i % B].cpu().numpy().tobytes(), args.k)
            ref = per_window.get((i % NH) % args.windows) if (i % NH) < args.windows else None
            if ref is not None and sdict is None:
                assert st_ == 0 and np.array_equal(ref[0], o_) and np.array_equal(ref[1], d_), "host-resident mismatch"
        for hw in hws:
            L.gf_window_destroy(hw)
        for pin in pins:
            L.gf_pinned_free(pin)
        wnd = breakdown.get("window_us", 0.0) * 1e-6
        pcie = {"bytes_per_window": bpp * n, "columns": "x, y, objID (ts not uploaded)",
                "upload_pinned_ms": round(1e3 * res["pinned"], 3),
                "upload_pageable_ms": round(1e3 * res["pageable"], 3),
                "upload_pinned_GBps": round(bpp * n / res["pinned"] / 1e9, 1),
                "serial_upload_then_evaluate_points_per_s": round(n / (res["pinned"] + wnd), 1),
                "host_resident_pipelined_points_per_s": round(n / hpipe, 1),
                "host_resident_pipelined_ms_per_window": round(1e3 * hpipe, 3),
                "host_resident_note": (f"{NH} distinct pinned host windows streamed through 2 device windows: "
                                       "upload(i+1) on the window's copy stream overlaps evaluate(i); PCIe-bound"),
                "host_resident_16B_points_per_s": round(n / hpipe16, 1),
                "host_resident_16B_ms_per_window": round(1e3 * hpipe16, 3),
                "host_resident_16B_note": ("gf_window_upload_mapped: x, y copied (16 B per point), the objID column "
                                           "read in place from pinned host memory (only the candidates' objIDs cross "
                                           "PCIe); records checked against the device-resident ones")}

    verified = None
    cpu = None
    if rank == 0 and world > 1 and not args.no_verify and world * n <= 100_000_000:
        # the merged record of window 0 (every rank's band of it, all-gathered over the
        # backend and merged on the device) == the oracle on the whole window: rank 0
        # regenerates the other ranks' bands (same seeds) and concatenates them in rank order,
        # so the global index of rank r's point i is r * n + i (its plan's index base)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        t = time.perf_counter()
        xs, ys, objs = [], [], []
        for r_ in range(world):
            blo, bhi = sharding.column_bands(args.grid, world)[r_]
            bx0, bx1 = sharding.band_x_range(grid, blo, bhi)
            x_, y_ = W.gen_points(sf, 42 + 1000 * r_, n, bx0, bx1)
            xs.append(x_); ys.append(y_); objs.append(np.arange(r_ * n, (r_ + 1) * n, dtype=np.int64))
        og = O.grid(args.grid, *BEIJING)
        st, oo, od, oi = O.knn(og, np.concatenate(xs), np.concatenate(ys), np.concatenate(objs), QPOINT[0],
                               QPOINT[1], args.radius, args.k)
        got = per_window[0]
        verified = bool(st == 0 and np.array_equal(oo, got[0]) and np.array_equal(od, got[1])
                        and np.array_equal(oi, got[2]))
        log(f"oracle verification of window 0 over {world} ranks x {n} points: {verified} "
            f"({time.perf_counter()-t:.1f}s)")
        assert verified, "merged multi-rank kNN differs from the oracle"
    if rank == 0 and world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        og = O.grid(args.grid, *BEIJING)
        if not args.no_verify:
            t = time.perf_counter()
            verified = True
            for j, (x, y, obj) in enumerate(host_windows):
                st, oo, od, oi = O.knn(og, x, y, obj, QPOINT[0], QPOINT[1], args.radius, args.k)
                got = per_window[j]
                verified &= bool(st == 0 and np.array_equal(oo, got[0]) and np.array_equal(od, got[1])
                                 and np.array_equal(oi, got[2]))
            log(f"oracle verification of {len(host_windows)} windows: {verified} ({time.perf_counter()-t:.1f}s)")
            assert verified, "GPU kNN differs from the oracle"
        if not args.no_cpu_baseline:
            cpu = cpu_baselines(args, O, og, host_windows[0], per_window[0], n)

    traffic, traffic_src = None, None
    if rank == 0:  # HBM bytes per launch from the committed rocprofv3 PMC pass of this command
        import glob

        kname = "knn_fused" if args.pipeline >= 2 else "knn_scan"
        # newest round first: r<NN>_knn_pmc.json (tools/pmc_table.py: per-kernel medians) or the
        # older r<NN>_<kernel>_pmc.json (one kernel, FETCH_SIZE / WRITE_SIZE summaries)
        files = glob.glob(os.path.join(ROOT, "profiles", "r*_knn_pmc.json")) + \
            glob.glob(os.path.join(ROOT, "profiles", f"r*_{kname}_pmc.json"))
        for f in sorted(files, key=lambda f: os.path.basename(f).split("_")[0], reverse=True):
            with open(f) as fh:
                pm = json.load(fh)
            if "pmc" in pm:  # tools/pmc_table.py layout: the dominant kernel's entry
                ent = [v for k_, v in pm["pmc"].items() if f"{kname}_kernel" in k_]
                if ent and "hbm_read_bytes_corrected" in ent[0]:
                    traffic = ent[0]["hbm_read_bytes_corrected"] + ent[0].get("hbm_write_bytes", 0.0)
                    traffic_src = (os.path.relpath(f, ROOT) + f": rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes, "
                                   f"median per {kname}_kernel launch, FETCH_SIZE x2 (gfx950)")
                    break
            elif pm.get("points_per_launch", n) == n and "FETCH_SIZE" in pm:
                traffic = pm["FETCH_SIZE"]["corrected_bytes_per_launch"] + 1024.0 * pm["WRITE_SIZE"]["median_KB"]
                traffic_src = (os.path.relpath(f, ROOT) + ": rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes, "
                               "median per launch, FETCH_SIZE x2 (gfx950)")
                break

    if rank == 0:
        pts_per_step = world * n
        value = pts_per_step * args.steps / elapsed
        avg_scan_s = scan_ms / 1000.0 / max(scan_n, 1)
        bytes_per_launch = 16.0 * n  # x, y fp64 per point; objID read only for candidates
        # depth 3 keeps two launches in flight (one per stream), so a launch's own duration
        # overlaps its neighbour's: the kernel's sustained rate is then bytes per launch over the
        # launch interval (= ms_per_step, host included), not over one launch's duration
        in_flight = args.pipeline - 1 if args.pipeline >= 3 else 1
        interval_s = elapsed / args.steps if in_flight > 1 else avg_scan_s
        achieved = bytes_per_launch / interval_s / 1e9
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "points/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": (W.data_desc().replace(", device-resident", "") + f", {args.windows} distinct "
                     "device-resident windows cycled (continuous query)"),
            "config": {
                "workload": f"knn_k{args.k}_r{args.radius}_{n // 1_000_000}Mpts_per_gpu_grid{args.grid}x{args.grid}"
                            + ("_clustered" if args.clustered else ""),
                "points_per_window": pts_per_step,
                "points_per_gpu": n,
                "k": args.k,
                "radius": args.radius,
                "grid": args.grid,
                "query_point": list(QPOINT),
                "parallelism": f"cell-column shards x{world}" + (" + RCCL all-gather top-k" if world > 1 else ""),
                "windows_in_flight": args.pipeline,
                "exchange_batch": B if world > 1 else None,
                "exchange": xdesc,
                "objid": ("dictionary Strings" + (" (string records merged by String)" if world > 1 else ""))
                         if args.string_objids else "canonical decimal (int64 keys)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": {1: "knn_scan",
                           2: "knn_fused (scan of window i + select of window i-1 in block 0)",
                           3: "knn_fused (scan of window i + select of window i-2 in block 0; "
                              "consecutive windows on two streams)",
                           4: "knn_fused (scan of window i + select of window i-3 in block 0; "
                              "consecutive windows on three streams)"}[args.pipeline],
                "achieved_basis": (f"bytes per launch / launch interval ({in_flight} launches in flight)" if in_flight > 1
                                   else "bytes per launch / avg launch duration (HIP events)"),
                "launches_in_flight": in_flight,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "bytes_per_launch": bytes_per_launch,
                "avg_launch_us": round(avg_scan_s * 1e6, 2),
                "launches_timed": scan_n,
            },
            "cpu_baseline": cpu,
            "breakdown": breakdown,
            "host_boundary": pcie,
            "verified_vs_oracle": verified,
            "build": L.gf_build_info().decode(),
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.destroy()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
