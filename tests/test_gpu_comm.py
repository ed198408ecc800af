"""GPU: the RCCL exchange behind the C ABI (gf_comm_* + gf_knn_exchange_*), the windowAll funnel
across GPUs (PointPointKNNQuery.java:198-200 -> KNNQuery.java:213-272) the Java drop-in calls.
One MI355X per box, and RCCL refuses two ranks on one device, so the communicators here have one
rank: ncclCommInitRank (gf_comm_create) and ncclCommInitAll (gf_comm_create_all) -- the all-gather
and the device merge run through the library exactly as at N ranks, and the merged records must
equal the oracle on each window.  The multi-rank layout is checked with gloo ranks on the CPU
(tests/test_sharding_gloo.py) and bench.py's two-rank runs (tests/test_a_gpu_multirank.py)."""
import numpy as np
import pytest

from conftest import BEIJING, QPOINT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sf(gpu):
    import spatialflink_amd

    return spatialflink_amd


def _windows(oracle_mod, nwin, n):
    out = []
    for j in range(nwin):
        x, y = oracle_mod.java_random_points(70 + j, n, *BEIJING)
        obj = (np.random.default_rng(j).permutation(n) % max(1, n * 3 // 4)).astype(np.int64)
        out.append((x, y, obj))
    return out


def _records(sf, windows, k):
    """each window evaluated into a device record (gf_knn_enqueue at depth 1) -> [nwin, rb] uint8"""
    import torch

    g = sf.UniformGrid(500, *BEIJING)
    q = sf.Point("q", *QPOINT, 0, g)
    op = sf.PointPointKNNQuery(sf.QueryConfiguration(sf.QueryType.WindowBased), g)
    rb = sf.spatialOperators.knn_record_bytes(k)
    recs = torch.zeros(len(windows), rb, dtype=torch.uint8, device="cuda")
    keep = []
    for i, (x, y, obj) in enumerate(windows):
        w = sf.PointWindow.from_numpy(x, y, obj)
        keep.append(w)
        op.enqueue(w, q, 0.5, k, recs[i])
    op.flush(0, q, 0.5, k)
    torch.cuda.synchronize()
    return recs, keep


def _check(sf, oracle_mod, raw, k, x, y, obj):
    og = oracle_mod.grid(500, *BEIJING)
    st, o, d, i = sf.spatialOperators.decode_knn_record(raw, k)
    assert st == 0
    est, eo, ed, ei = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
    np.testing.assert_array_equal(o, eo)
    np.testing.assert_array_equal(d.view(np.int64), ed.view(np.int64))
    np.testing.assert_array_equal(i, ei)


def test_comm_available(sf):
    assert sf.sharding.Comm.available(), sf._lib.lib().gf_comm_last_error(None)


@pytest.mark.parametrize("k", [50, 600])
def test_knn_exchange_one_rank(sf, oracle_mod, k):
    import torch

    wins = _windows(oracle_mod, 3, 300_000)
    recs, keep = _records(sf, wins, k)
    comm = sf.sharding.Comm.single(0)
    try:
        assert (comm.nranks, comm.rank) == (1, 0)
        merged = torch.zeros_like(recs)
        comm.exchange_batch(recs, k, merged)
        # a second batch through the same (grown) gather buffer, into mapped pinned memory
        pinned = sf.PinnedRecords(len(wins), k)
        comm.exchange_batch(recs, k, pinned.ptr(0))
        torch.cuda.synchronize()
        assert sf._lib.lib().gf_comm_check(comm.handle) == 0
        for j, (x, y, obj) in enumerate(wins):
            _check(sf, oracle_mod, merged[j].cpu().numpy().tobytes(), k, x, y, obj)
            _check(sf, oracle_mod, pinned.raw(j), k, x, y, obj)
    finally:
        comm.destroy()


def test_knn_exchange_group_create_all(sf, oracle_mod):
    """ncclCommInitAll clique (one process driving its GPUs), exchanged as one RCCL group."""
    import torch

    k = 40
    wins = _windows(oracle_mod, 2, 200_000)
    recs, keep = _records(sf, wins, k)
    comms = sf.sharding.Comm.create_all([0])
    try:
        merged = torch.zeros_like(recs)
        ctx = sf._lib.context(0)
        sf.sharding.exchange_group(comms, [ctx], [recs], k, [merged])
        torch.cuda.synchronize()
        for j, (x, y, obj) in enumerate(wins):
            _check(sf, oracle_mod, merged[j].cpu().numpy().tobytes(), k, x, y, obj)
    finally:
        for c in comms:
            c.destroy()


def test_knn_exchange_strings_one_rank(sf, oracle_mod):
    """String objIDs: the records' dictionary Strings attached, all-gathered, merged by String."""
    import torch

    k, cap = 30, 16 * 30 + 64
    wins = _windows(oracle_mod, 2, 200_000)
    sdict = sf.ObjIdDict(0)
    dev_wins, keyed = [], []
    for x, y, obj in wins:
        strs = [b"veh%09d" % v for v in obj.tolist()]
        offs = np.zeros(len(strs) + 1, np.int64)
        offs[1:] = np.cumsum([len(s_) for s_ in strs])
        keys = np.empty(len(strs), np.int64)
        sf._lib.check(sf._lib.lib().gf_objid_intern(sdict.handle, b"".join(strs), offs.ctypes.data, len(strs),
                                                    keys.ctypes.data), sdict.ctx.handle, "intern")
        keyed.append((x, y, keys))
    recs, keep = _records(sf, keyed, k)
    comm = sf.sharding.Comm.single(0)
    try:
        sb = sf.sharding.string_record_bytes(k, cap)
        merged = torch.zeros(len(wins), sb, dtype=torch.uint8, device="cuda")
        comm.exchange_strings_batch(recs, k, cap, sdict, merged)
        torch.cuda.synchronize()
        og = oracle_mod.grid(500, *BEIJING)
        for j, (x, y, obj) in enumerate(wins):
            st, strs, d, ix = sf.sharding.decode_string_record(merged[j].cpu().numpy().tobytes(), k, cap)
            assert st == 0
            est, eo, ed, ei = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], 0.5, k)
            # "veh%09d" orders like its number: the oracle on the integers is the String contract
            assert [int(s_[3:]) for s_ in strs] == eo.tolist()
            np.testing.assert_array_equal(d.view(np.int64), ed.view(np.int64))
            np.testing.assert_array_equal(ix, ei)
    finally:
        comm.destroy()
