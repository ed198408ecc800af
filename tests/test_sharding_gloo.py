"""CPU, world_size 2 (gloo): the multi-GPU decomposition -- cell-column shards, concatenated
range hits, all-gathered kNN top-k merge, halo-replicated join -- reproduces the
single-window result.  The per-shard evaluator here is the oracle (no GPU in this
container); the GPU per-shard kernels are covered by tests/test_gpu_parity.py."""
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

        # kNN: per-shard top-k (global indices), all-gather, merge
        for r, k in ((0.5, 50), (0.05, 20), (0.3, 200)):
            st, o, d, i = O.knn(og, x[idx], y[idx], obj[idx], QPOINT[0], QPOINT[1], r, k)
            mo, md, mi = sharding.allgather_knn_lists(o, d, idx[i], k)
            st, fo, fd, fi = O.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
            assert np.array_equal(mo, fo) and np.array_equal(md, fd) and np.array_equal(mi, fi), (r, k)

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
