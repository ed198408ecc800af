"""CPU, world_size 2 (gloo): the host side of the multi-GPU decomposition -- cell-column band
arithmetic, the kNN record exchange (sharding.gather_records_batch: the same all_gather of
[nwin, rb] byte records the RCCL path runs, here over gloo on CPU tensors, decoded in the
shard-major layout gf_knn_merge_dev_batch reads, merged with the library's host merge),
concatenated range hits and the halo-replicated join.  The shard results fed in are the
oracle's (no GPU here); the product kernels per shard and the device merge are covered by
tests/test_gpu_sharding.py on the GPU."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import BEIJING, QPOINT, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ret):
    import sys

    for p in (ROOT, os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle as O

    from spatialflink_amd import sharding

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 500
        og = O.grid(n, *BEIJING)
        x, y = O.java_random_points(5, 60_000, 115.4, 117.7, 39.5, 41.2)
        obj = (np.arange(len(x)) * 7 % 50_000).astype(np.int64)  # duplicated objIDs on purpose
        cx, cy = O.assign_cells(og, x, y)
        col_counts = np.bincount(np.clip(cx, 0, n - 1), minlength=n)
        bands = sharding.column_bands(n, world, col_counts)
        own = sharding.shard_of_columns(cx, bands) == rank
        idx = np.nonzero(own)[0]

        # kNN: per-shard top-k records of 3 windows (global indices) in ONE all-gather of byte
        # records, decoded shard-major, merged per window
        import torch
        from spatialflink_amd.spatialOperators import decode_knn_record, knn_merge_host, knn_record_bytes

        for r, k in ((0.5, 50), (0.05, 20), (0.3, 200)):
            rb = knn_record_bytes(k)
            nwin = 3
            recs = torch.zeros(nwin, rb, dtype=torch.uint8)
            for w in range(nwin):
                sel = idx[w:]  # windows differ: drop the first w points of the shard
                st, o, d, i = O.knn(og, x[sel], y[sel], obj[sel], QPOINT[0], QPOINT[1], r, k)
                recs[w] = torch.frombuffer(bytearray(sharding.encode_knn_record(k, o, d, sel[i])), dtype=torch.uint8)
            gathered = sharding.gather_records_batch(recs).numpy()
            assert gathered.size == world * nwin * rb
            for w in range(nwin):
                lists = []
                for s_ in range(world):  # record (shard s, window w) at (s * nwin + w) * rb
                    st, o, d, i = decode_knn_record(gathered[(s_ * nwin + w) * rb:(s_ * nwin + w + 1) * rb].tobytes(), k)
                    assert st == 0
                    lists.append((o, d, i))
                mo, md, mi = knn_merge_host(k, lists)
                keep = np.ones(len(x), bool)
                for s_ in range(world):  # the window: every rank dropped its own first w points
                    keep[np.nonzero(sharding.shard_of_columns(cx, bands) == s_)[0][:w]] = False
                al = np.nonzero(keep)[0]
                st, fo, fd, fi = O.knn(og, x[al], y[al], obj[al], QPOINT[0], QPOINT[1], r, k)
                assert np.array_equal(mo, fo) and np.array_equal(md, fd) and np.array_equal(mi, al[fi]), (r, k, w)
            mo, md, mi = sharding.allgather_knn_lists(*O.knn(og, x[idx], y[idx], obj[idx], QPOINT[0], QPOINT[1], r, k)[1:3],
                                                      idx[O.knn(og, x[idx], y[idx], obj[idx], QPOINT[0], QPOINT[1], r, k)[3]], k)
            st, fo, fd, fi = O.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
            assert np.array_equal(mo, fo) and np.array_equal(md, fd) and np.array_equal(mi, fi), (r, k)
            # String objIDs (dictionary keys are per-rank ids): the exchange carries the Strings
            name = lambda v: f"bus-{v:05d}"  # noqa: E731  (non-numeric: dictionary Strings on a device)
            st, so_, sd_, si_ = O.knn(og, x[idx], y[idx], obj[idx], QPOINT[0], QPOINT[1], r, k)
            mo, md, mi = sharding.allgather_knn_string_lists([name(v) for v in so_], sd_, idx[si_], k)
            assert mo == [name(v).encode() for v in fo] and np.array_equal(md, fd) and np.array_equal(mi, fi), (r, k)

        # range: per-shard hits, concatenated
        for r in (0.5, 0.05):
            hits = idx[O.range_pp(og, x[idx], y[idx], [QPOINT[0]], [QPOINT[1]], r)]
            allh = [None] * world
            dist.all_gather_object(allh, hits)
            got = np.sort(np.concatenate(allh))
            assert np.array_equal(got, O.range_pp(og, x, y, [QPOINT[0]], [QPOINT[1]], r)), r

        # join: ordinary side sharded by columns, query side replicated with a c-column halo
        qx, qy = O.java_random_points(6, 6_000, 115.4, 117.7, 39.5, 41.2)
        qcx, _ = O.assign_cells(og, qx, qy)
        for r in (0.001, 0.01):
            c = O.layers(og, r)[1]
            qm = sharding.join_query_halo(qcx, bands[rank], c)
            qi = np.nonzero(qm)[0]
            st, pairs = O.join_pp(og, og, x[idx], y[idx], qx[qi], qy[qi], r)
            mine = np.stack([idx[pairs[:, 0]], qi[pairs[:, 1]]], 1) if len(pairs) else np.zeros((0, 2), np.int64)
            allp = [None] * world
            dist.all_gather_object(allp, mine)
            got = sorted(map(tuple, np.concatenate(allp).tolist()))
            st, full = O.join_pp(og, og, x, y, qx, qy, r)
            assert got == sorted(map(tuple, full.tolist())), r
        ret[rank] = "ok"
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_decomposition(oracle_mod):
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.start_processes(_worker, args=(world, port, ret), nprocs=world, join=True, start_method="spawn")
    assert dict(ret) == {0: "ok", 1: "ok"}


def test_column_bands_balance():
    from spatialflink_amd import sharding

    assert sharding.column_bands(500, 8) == [((r * 500) // 8, ((r + 1) * 500) // 8) for r in range(8)]
    counts = np.zeros(100)
    counts[:10] = 1000.0
    counts[10:] = 1.0
    b = sharding.column_bands(100, 4, counts)
    assert b[0][0] == 0 and b[-1][1] == 100 and all(b[i][1] == b[i + 1][0] for i in range(3))
    assert b[0][1] <= 4  # the dense columns are split across ranks
