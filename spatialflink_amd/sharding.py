"""Multi-GPU evaluation of one window: points sharded by grid-cell column ranges across the
GPUs of one node (one process per GPU, torch.distributed over RCCL/xGMI).

The reference distributes by keyBy(gridID) (hash of the cell string) over Flink subtasks
(PointPointRangeQuery.java:144-148) and funnels kNN through a parallelism-1 windowAll
(PointPointKNNQuery.java:198-200).  Here each rank owns a contiguous band of cell columns;
range hits need no exchange (concatenate), kNN needs one all-gather of k x (dist, objID, idx)
records followed by the same deterministic top-k-distinct merge on every rank.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


def column_bands(n_cols: int, world: int, col_counts=None):
    """Cell-column ranges [lo, hi) per rank.  With a per-column point histogram the bands
    balance point counts (the bucketing histogram doubles as the load balancer); without
    one they split the columns evenly."""
    if col_counts is None:
        edges = [(r * n_cols) // world for r in range(world + 1)]
    else:
        c = np.cumsum(np.asarray(col_counts, np.float64))
        total = c[-1] if len(c) else 0.0
        edges = [0]
        for r in range(1, world):
            edges.append(int(np.searchsorted(c, total * r / world)) + 1)
        edges.append(n_cols)
        for i in range(1, len(edges)):
            edges[i] = max(edges[i], edges[i - 1])
    return [(edges[r], edges[r + 1]) for r in range(world)]


def work_bands(n_cols: int, world: int, col_points, col_candidates=None, candidate_cost: float = 0.0):
    """Bands balanced by WORK, not points: every point costs its 16-B scan, a point the plan
    queues for the exact test (a candidate-cell point of a polygon set, C3) costs
    `candidate_cost` scans more.  Without candidates this is column_bands(col_points)."""
    w = np.asarray(col_points, np.float64)
    if col_candidates is not None:
        w = w + candidate_cost * np.asarray(col_candidates, np.float64)
    return column_bands(n_cols, world, w)


def _hit_cells(grid, bboxes, r):
    """[n, n] (row-major by cy): cells touched by some query object's bbox expanded by r."""
    n = grid.getNumGridPartitions()
    cl = grid.getCellLength()
    hit = np.zeros((n, n), dtype=bool)
    for x1, y1, x2, y2 in np.asarray(bboxes, np.float64):
        a0 = max(int(np.floor((x1 - r - grid.getMinX()) / cl)), 0)
        a1 = min(int(np.floor((x2 + r - grid.getMinX()) / cl)), n - 1)
        b0 = max(int(np.floor((y1 - r - grid.getMinY()) / cl)), 0)
        b1 = min(int(np.floor((y2 + r - grid.getMinY()) / cl)), n - 1)
        if a0 <= a1 and b0 <= b1:
            hit[b0:b1 + 1, a0:a1 + 1] = True
    return hit


def candidate_cells_per_column(grid, bboxes, r):
    """Per-column number of cells the plan tests exactly: with uniform points, the expected
    candidate term of work_bands is this times the points per cell."""
    return _hit_cells(grid, bboxes, r).sum(axis=0)


def candidate_columns(grid, cx, cy, bboxes, r):
    """Per-column count of the points that lie in a cell touched by some query object's bbox
    expanded by r (the cells a range / join plan tests exactly) -- the candidate term of
    work_bands.  bboxes: [m, 4] (x1, y1, x2, y2)."""
    n = grid.getNumGridPartitions()
    hit = _hit_cells(grid, bboxes, r)
    cx = np.asarray(cx, np.int64)
    cy = np.asarray(cy, np.int64)
    ok = (cx >= 0) & (cy >= 0) & (cx < n) & (cy < n)
    cand = np.zeros(len(cx), dtype=bool)
    cand[ok] = hit[cy[ok], cx[ok]]
    return np.bincount(cx[cand], minlength=n)[:n]


def shard_order(cx, bands):
    """A window's points grouped by owning rank, arrival order kept inside a shard:
    (perm, offsets) with shard s = perm[offsets[s]:offsets[s+1]] (global point indices) -- a
    rank's window is that slice, and its kNN index base is offsets[s] in the permuted order."""
    owner = shard_of_columns(np.asarray(cx, np.int64), bands)
    perm = np.argsort(owner, kind="stable")
    offsets = np.searchsorted(owner[perm], np.arange(len(bands) + 1), side="left")
    return perm, offsets


def shard_window(window, grid, bands):
    """The device form of shard_order for an arriving window (gf_shard_by_columns): the window's
    points grouped by owning band, arrival order kept inside a band -> (perm: torch uint32 as
    int32 [n], offsets: numpy int64 [len(bands) + 1]); band s = perm[offsets[s]:offsets[s+1]]."""
    import torch

    ctx = _lib.context(window.x.device.index)
    n = window.n
    lo = np.ascontiguousarray([b[0] for b in bands], np.int32)
    perm = torch.empty(max(n, 1), dtype=torch.int32, device=window.x.device)
    off = torch.empty(len(bands) + 1, dtype=torch.int32, device=window.x.device)
    pts = window.c_struct()
    _lib.check(_lib.lib().gf_shard_by_columns(ctx.handle, C.byref(grid.c_grid), C.byref(pts), len(bands),
                                              lo.ctypes.data, perm.data_ptr(), off.data_ptr()),
               ctx.handle, "gf_shard_by_columns")
    return perm[:n], off.cpu().numpy().view(np.uint32).astype(np.int64)


def gather_shard(window, perm, offsets, s):
    """Band s of a window routed by shard_window as its own PointWindow (gf_gather_points): the
    SoA slice a rank receives."""
    import torch

    from .spatialObjects import PointWindow

    ctx = _lib.context(window.x.device.index)
    b, e = int(offsets[s]), int(offsets[s + 1])
    dev = window.x.device
    out = [torch.empty(max(e - b, 1), dtype=dt, device=dev) for dt in (torch.float64, torch.float64, torch.int64,
                                                                        torch.int64)]
    pts = window.c_struct()
    _lib.check(_lib.lib().gf_gather_points(ctx.handle, C.byref(pts), perm.data_ptr(), b, e, *(t.data_ptr() for t in out)),
               ctx.handle, "gf_gather_points")
    return PointWindow(*(t[: e - b] for t in out))


def band_x_range(grid, lo: int, hi: int):
    """Coordinate range covering cell columns [lo, hi) (for generating a rank's shard)."""
    return grid.getMinX() + lo * grid.getCellLength(), grid.getMinX() + hi * grid.getCellLength()


def shard_of_columns(cx: np.ndarray, bands) -> np.ndarray:
    """Rank owning each point's column; out-of-grid columns go to the nearest edge rank."""
    lows = np.array([b[0] for b in bands])
    r = np.searchsorted(lows, cx, side="right") - 1
    return np.clip(r, 0, len(bands) - 1)


def merge_knn_records_host(records, k: int):
    """Top-k-distinct merge of per-shard records (host bytes) -> (objID, dist, idx)."""
    from .spatialOperators import decode_knn_record, knn_merge_host

    lists = []
    for raw in records:
        st, o, d, i = decode_knn_record(raw, k)
        if st != 0:
            raise _lib.GeoFlinkError(_lib.GF_ERR_HIP, "shard record needs the exact fallback; decode it first")
        lists.append((o, d, i))
    return knn_merge_host(k, lists)


def allgather_knn_lists(objID, dist, idx, k: int, group=None):
    """Any backend (gloo on CPU too): all_gather_object of this rank's sorted list, then the
    deterministic top-k-distinct merge.  Identical result on every rank."""
    import torch.distributed as dist_

    world = dist_.get_world_size(group)
    mine = (np.asarray(objID, np.int64), np.asarray(dist, np.float64), np.asarray(idx, np.int64))
    gathered = [None] * world
    dist_.all_gather_object(gathered, mine, group=group)
    from .spatialOperators import knn_merge_host

    return knn_merge_host(k, gathered)


def _all_gather_bytes(out, inp, group):
    """all_gather_into_tensor; device tensors go through host memory on gloo (CPU rehearsal
    of the multi-rank path on one GPU), straight over RCCL otherwise."""
    import torch.distributed as dist_

    if inp.is_cuda and dist_.get_backend(group) == "gloo":
        tmp = out.cpu()
        dist_.all_gather_into_tensor(tmp, inp.cpu(), group=group)
        out.copy_(tmp)
    else:
        dist_.all_gather_into_tensor(out, inp, group=group)


def _merge_layout(world: int) -> int:
    """Shard-major; with more than one rank the records come from other ranks' contexts, whose
    dictionary objID keys cannot be compared (GF_MERGE_FOREIGN_KEYS).  A one-rank group's records
    all come from this context's own dictionary and merge as is."""
    return _lib.GF_MERGE_SHARD_MAJOR | (_lib.GF_MERGE_FOREIGN_KEYS if world > 1 else 0)


def allgather_knn_records(record, k: int, merged_out, group=None):
    """RCCL path: all-gather this rank's device kNN record (uint8 tensor of
    knn_record_bytes(k)) over xGMI, then merge the world's records on the device
    (gf_knn_merge_dev) into `merged_out` (a device tensor, or an int address from
    PinnedRecords.ptr()).  Stream-ordered, no host sync."""
    import torch
    import torch.distributed as dist_

    world = dist_.get_world_size(group)
    rb = record.numel()
    gathered = torch.empty(world * rb, dtype=torch.uint8, device=record.device)
    _all_gather_bytes(gathered, record, group)
    ctx = _lib.context(record.device.index)
    out = merged_out if isinstance(merged_out, int) else merged_out.data_ptr()
    _lib.check(_lib.lib().gf_knn_merge_dev_batch(ctx.handle, int(k), gathered.data_ptr(), world, 1,
                                                 _merge_layout(world), out),
               ctx.handle, "gf_knn_merge_dev_batch")
    return merged_out


def gather_records_batch(records, group=None):
    """The collective of allgather_knn_records_batch: this rank's [nwin, rb] uint8 records ->
    the world's, shard-major ([world * nwin * rb]: rank s's window w at (s * nwin + w) * rb) --
    the layout gf_knn_merge_dev_batch(GF_MERGE_SHARD_MAJOR) reads.  CPU tensors over gloo too."""
    import torch
    import torch.distributed as dist_

    world = dist_.get_world_size(group)
    nwin, rb = records.shape
    gathered = torch.empty(world * nwin * rb, dtype=torch.uint8, device=records.device)
    _all_gather_bytes(gathered, records.reshape(-1), group)
    return gathered


def encode_knn_record(k: int, objID, dist, idx, status: int = 0, candidates: int = 0, threshold: float = 0.0):
    """Host bytes of a kNN result record (gf_knn_header + dist[k] + objID[k] + idx[k]) -- the
    inverse of spatialOperators.decode_knn_record (for host-side shards and tests)."""
    n = len(objID)
    h = _lib.GfKnnHeader(int(status), n, int(k), 0, int(candidates), float(threshold))
    d = np.zeros(k, np.float64); o = np.zeros(k, np.int64); i = np.zeros(k, np.int64)
    d[:n] = dist; o[:n] = objID; i[:n] = idx
    return bytes(h) + d.tobytes() + o.tobytes() + i.tobytes()


def allgather_knn_records_batch(records, k: int, results, group=None, ctx=None):
    """One RCCL all-gather for several windows: `records` is this rank's [nwin, rb] uint8
    device tensor (consecutive windows); every rank merges all windows in one launch
    (gf_knn_merge_dev_batch, shard-major) into `results` -- nwin consecutive records (device
    tensor or an int address from PinnedRecords.ptr()).  Stream-ordered, no host sync.
    Batching amortises the collective's latency over nwin windows (xGMI is point to point:
    small messages are latency-, not bandwidth-bound).

    objID keys: canonical decimal objIDs are their values on every rank and merge as is.  A
    dictionary key (a non-numeric String objID) is an id in its own rank's gf_objid_dict, so
    keys of different ranks cannot be compared: the merge refuses such a window (record status
    _lib.KNN_STATUS_FOREIGN_KEYS, no entries) -- merge those on the device by their Strings with
    allgather_knn_records_strings.

    Ordering (pipeline depth 3): odd windows' records are written on the plan's second stream.
    Before this call, gf_ctx_join (the context stream waits for the second stream) so the
    records are complete; after it, gf_ctx_fork (the second stream waits for the context
    stream) before `records` is handed to later enqueues, so no later window overwrites them
    while the all-gather still reads them.

    ctx: the context whose stream runs the merge (default: the thread's context, bound to
    torch's current stream).  An exchange overlapped with the next windows runs under
    `torch.cuda.stream(side)` with a context of its own bound to that side stream -- the thread's
    cached context (the plan's) must not be rebound to it."""
    import torch.distributed as dist_

    world = dist_.get_world_size(group)
    nwin = records.shape[0]
    gathered = gather_records_batch(records, group)
    if ctx is None:
        ctx = _lib.context(records.device.index)
    out = results if isinstance(results, int) else results.data_ptr()
    _lib.check(_lib.lib().gf_knn_merge_dev_batch(ctx.handle, int(k), gathered.data_ptr(), world, int(nwin),
                                                 _merge_layout(world), out),
               ctx.handle, "gf_knn_merge_dev_batch")
    return results


class Comm:
    """An RCCL communicator behind the C ABI (gf_comm_*): the transport of the kNN record exchange
    the Java drop-in uses, so the exchange measured by bench.py is the same code.

    Comm.from_group(device): one process per GPU -- rank 0's gf_comm_unique_id goes to every rank
    over the job's control plane (torch.distributed broadcast_object_list: gloo or nccl), then
    gf_comm_create (ncclCommInitRank).  Comm.single(device): a one-rank communicator.
    Comm.create_all(devices): one process driving several GPUs (ncclCommInitAll)."""

    def __init__(self, handle, device: int):
        self.handle = handle
        self.device = int(device)
        n, r, d = C.c_int32(), C.c_int32(), C.c_int()
        _lib.check(_lib.lib().gf_comm_info(handle, C.byref(n), C.byref(r), C.byref(d)), None, "gf_comm_info")
        self.nranks, self.rank = n.value, r.value

    @staticmethod
    def available() -> bool:
        return bool(_lib.lib().gf_comm_available())

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * _lib.GF_COMM_ID_BYTES)()
        st = _lib.lib().gf_comm_unique_id(buf)
        if st:
            raise _lib.GeoFlinkError(st, "gf_comm_unique_id: " + (_lib.lib().gf_comm_last_error(None) or b"").decode())
        return bytes(buf)

    @classmethod
    def create(cls, uid: bytes, nranks: int, rank: int, device: int) -> "Comm":
        h = C.c_void_p()
        idb = (C.c_uint8 * _lib.GF_COMM_ID_BYTES).from_buffer_copy(uid)
        st = _lib.lib().gf_comm_create(idb, int(nranks), int(rank), int(device), C.byref(h))
        if st:
            raise _lib.GeoFlinkError(st, "gf_comm_create: " + (_lib.lib().gf_comm_last_error(None) or b"").decode())
        return cls(h, device)

    @classmethod
    def single(cls, device: int) -> "Comm":
        return cls.create(cls.unique_id(), 1, 0, device)

    @classmethod
    def from_group(cls, device: int, group=None) -> "Comm":
        import torch.distributed as dist_

        obj = [cls.unique_id() if dist_.get_rank(group) == 0 else None]
        dist_.broadcast_object_list(obj, src=0, group=group)
        return cls.create(obj[0], dist_.get_world_size(group), dist_.get_rank(group), device)

    @classmethod
    def create_all(cls, devices):
        devs = (C.c_int * len(devices))(*devices)
        hs = (C.c_void_p * len(devices))()
        st = _lib.lib().gf_comm_create_all(len(devices), devs, hs)
        if st:
            raise _lib.GeoFlinkError(st, "gf_comm_create_all: " + (_lib.lib().gf_comm_last_error(None) or b"").decode())
        return [cls(C.c_void_p(h), d) for h, d in zip(hs, devices)]

    def check(self, st, ctx, what):
        if st:
            detail = (_lib.lib().gf_comm_last_error(self.handle) or b"").decode()
            _lib.check(st, ctx, f"{what}: {detail}" if detail else what)

    def exchange_batch(self, records, k: int, results, ctx=None):
        """gf_knn_exchange_batch: this rank's [nwin, rb] uint8 device records -> nwin merged records
        (`results`: device tensor or an int address of mapped pinned memory), identical on every
        rank.  Async on ctx's stream (default: the thread's context)."""
        if ctx is None:
            ctx = _lib.context(records.device.index)
        out = results if isinstance(results, int) else results.data_ptr()
        self.check(_lib.lib().gf_knn_exchange_batch(self.handle, ctx.handle, int(k), records.data_ptr(),
                                                    int(records.shape[0]), out), ctx.handle, "gf_knn_exchange_batch")
        return results

    def exchange_strings_batch(self, records, k: int, cap_bytes: int, dictionary, results):
        """gf_knn_exchange_strings_batch: the String-objID form (records carry their Strings)."""
        out = results if isinstance(results, int) else results.data_ptr()
        self.check(_lib.lib().gf_knn_exchange_strings_batch(self.handle, dictionary.handle, int(k), int(cap_bytes),
                                                            records.data_ptr(), int(records.shape[0]), out),
                   dictionary.ctx.handle, "gf_knn_exchange_strings_batch")
        return results

    def destroy(self):
        if self.handle:
            _lib.lib().gf_comm_destroy(self.handle)
            self.handle = None


def open_comm(device: int, backend: str, mode: str = "auto", group=None):
    """The N > 1 kNN exchange's transport -> (Comm or None, description).  mode "rccl": the C ABI's
    communicator (gf_comm_create over the group's ranks) -- what the Java drop-in uses; "torch":
    torch.distributed's all_gather_into_tensor + gf_knn_merge_dev_batch; "auto": rccl on the nccl
    backend, torch on gloo (several ranks on one GPU, where RCCL refuses a duplicate device), and
    torch -- reported in the description -- if the communicator cannot be built."""
    if mode == "torch" or (mode == "auto" and backend != "nccl"):
        return None, "torch.distributed all_gather_into_tensor + gf_knn_merge_dev_batch"
    try:
        c = Comm.from_group(device, group)
        return c, "gf_knn_exchange_batch (RCCL ncclAllGather through the C ABI + gf_knn_merge_dev_batch)"
    except Exception as e:  # noqa: BLE001
        if mode == "rccl":
            raise
        return None, f"torch.distributed all_gather_into_tensor (gf_comm_create failed: {e})"


def exchange_group(comms, ctxs, records, k: int, results):
    """gf_knn_exchange_group: one thread drives every communicator of a create_all clique."""
    n = len(comms)
    hc = (C.c_void_p * n)(*[c.handle.value if isinstance(c.handle, C.c_void_p) else c.handle for c in comms])
    hx = (C.c_void_p * n)(*[x.handle.value if isinstance(x.handle, C.c_void_p) else x.handle for x in ctxs])
    rp = (C.c_void_p * n)(*[r.data_ptr() for r in records])
    op = (C.c_void_p * n)(*[o if isinstance(o, int) else o.data_ptr() for o in results])
    st = _lib.lib().gf_knn_exchange_group(n, hc, hx, int(k), rp, int(records[0].shape[0]), op)
    comms[0].check(st, ctxs[0].handle, "gf_knn_exchange_group")
    return results


def string_record_bytes(k: int, cap_bytes: int) -> int:
    """Bytes of a string record (a kNN record + the Strings of its dictionary objIDs)."""
    return int(_lib.lib().gf_knn_string_record_bytes(int(k), int(cap_bytes)))


def attach_strings(records, k: int, cap_bytes: int, dictionary, out=None):
    """gf_knn_attach_strings: this rank's [nwin, rb] device records -> [nwin, sb] string records
    carrying the Strings of their dictionary objIDs from `dictionary` (an ObjIdDict; async)."""
    import torch

    nwin = records.shape[0]
    sb = string_record_bytes(k, cap_bytes)
    if out is None:
        out = torch.empty((nwin, sb), dtype=torch.uint8, device=records.device)
    _lib.check(_lib.lib().gf_knn_attach_strings(dictionary.handle, int(k), records.data_ptr(), int(nwin),
                                                int(cap_bytes), out.data_ptr()), dictionary.ctx.handle,
               "gf_knn_attach_strings")
    return out


def allgather_knn_records_strings(records, k: int, cap_bytes: int, dictionary, results, group=None):
    """The device path of a String-objID kNN across ranks (KNNQuery.java:232-251 dedupes by
    String.equals): this rank's [nwin, rb] device records get their dictionary Strings attached
    (gf_knn_attach_strings), ONE all-gather carries the string records of every rank, and every
    rank merges all windows in one launch (gf_knn_merge_dev_strings, shard-major) into `results`
    -- nwin consecutive string records (device tensor, or an int address of pinned memory).
    Stream-ordered, no host sync; decode with decode_string_record.  The merge orders by
    (d, String bytes, idx) and dedupes by String, so every rank gets the same records."""
    import torch.distributed as dist_

    world = dist_.get_world_size(group)
    nwin = records.shape[0]
    ext = attach_strings(records, k, cap_bytes, dictionary)
    gathered = gather_records_batch(ext, group)
    ctx = _lib.context(records.device.index)
    out = results if isinstance(results, int) else results.data_ptr()
    _lib.check(_lib.lib().gf_knn_merge_dev_strings(ctx.handle, int(k), int(cap_bytes), gathered.data_ptr(), world,
                                                   int(nwin), _lib.GF_MERGE_SHARD_MAJOR, out),
               ctx.handle, "gf_knn_merge_dev_strings")
    return results


def decode_string_record(raw: bytes, k: int, cap_bytes: int):
    """Host bytes of a string record -> (status, [String bytes], dist, idx)
    (gf_knn_string_record_decode: dictionary Strings from the sidecar, Long.toString for decimals)."""
    import ctypes as C

    raw = bytes(raw)
    rec = C.create_string_buffer(raw, len(raw))
    st, n = C.c_int32(), C.c_int32()
    d = np.zeros(k, np.float64); i = np.zeros(k, np.int64); offs = np.zeros(k + 1, np.int64)
    cap = max(64, len(raw))
    for _ in range(2):
        buf = C.create_string_buffer(cap)
        rc = _lib.lib().gf_knn_string_record_decode(rec, int(k), int(cap_bytes), C.byref(st), None, d.ctypes.data,
                                                    i.ctypes.data, buf, cap, offs.ctypes.data, C.byref(n))
        if rc == _lib.GF_ERR_CAPACITY:
            cap = int(offs[n.value]) + 1
            continue
        _lib.check(rc, None, "gf_knn_string_record_decode")
        b = buf.raw
        m = n.value
        return st.value, [b[offs[j]:offs[j + 1]] for j in range(m)], d[:m].copy(), i[:m].copy()
    raise _lib.GeoFlinkError(_lib.GF_ERR_CAPACITY, "gf_knn_string_record_decode")


def merge_string_lists(k: int, lists):
    """Top-k-distinct merge of per-shard lists whose objIDs are Strings (bytes): sorted by
    (dist, objID String bytes), one entry per String (its minimum (dist, idx) occurrence), first
    k.  The rank-independent order for objIDs that are dictionary Strings: a dictionary key is an
    id in its own rank's dictionary, so only the Strings themselves compare across ranks (ties
    at exactly equal distances are ordered by the String's bytes)."""
    ent = []
    for objs, dist, idx in lists:
        ent += [(float(d), bytes(o), int(i)) for o, d, i in zip(objs, dist, idx)]
    ent.sort(key=lambda e: (e[0], e[1], e[2]))
    seen, out = set(), []
    for d, o, i in ent:
        if o in seen:
            continue
        seen.add(o)
        out.append((o, d, i))
        if len(out) == k:
            break
    return [e[0] for e in out], np.array([e[1] for e in out], np.float64), np.array([e[2] for e in out], np.int64)


def allgather_knn_string_lists(objid_strings, dist, idx, k: int, group=None):
    """kNN exchange for windows whose objIDs are dictionary Strings (keys of
    different ranks' dictionaries cannot be merged as integers).  Each rank decodes its sorted
    list's keys to Strings (PointWindow.objid_strings / ObjIdDict.decode_bytes), the lists are
    all-gathered (any backend) and merged by merge_string_lists -- identical on every rank.
    Intern the merged Strings into a rank's own dictionary to get its keys back."""
    import torch.distributed as dist_

    world = dist_.get_world_size(group)
    mine = ([o.encode() if isinstance(o, str) else bytes(o) for o in objid_strings],
            np.asarray(dist, np.float64), np.asarray(idx, np.int64))
    gathered = [None] * world
    dist_.all_gather_object(gathered, mine, group=group)
    return merge_string_lists(k, gathered)


def join_query_halo(qcx: np.ndarray, band, c: int) -> np.ndarray:
    """Query points a rank needs for its ordinary band [lo, hi): those whose cell column is
    within c = ceil(r / cellLength) of the band (the replicated-key neighbourhood,
    JoinQuery.java:73-90).  c < 0 (r == 0: every cell is a neighbour) -> all of them.
    Each pair (p, q) is then produced exactly once, by p's owner."""
    lo, hi = band
    if c < 0:
        return np.ones(len(qcx), dtype=bool)
    qcx = np.asarray(qcx, np.int64)
    return (qcx >= lo - c) & (qcx <= hi - 1 + c)
