"""CPU: sliding-window host logic -- Flink window assignment vs pane geometry, and the pane
decomposition the device engine relies on (top-k-distinct of a window == merge of its panes'
top-k-distinct lists), checked with the oracle and the library's host merge."""
import numpy as np
import pytest

from conftest import BEIJING, QPOINT


@pytest.mark.parametrize("size,slide", [(10_000, 5_000), (3_000, 1_000), (3_000, 2_000), (7_000, 7_000),
                                        (5_000, 3_000)])
def test_window_assignment_matches_panes(size, slide):
    from spatialflink_amd.windows import SlidingWindows

    g = SlidingWindows(size, slide)
    assert g.pane == np.gcd(size, slide)
    for ts in list(range(-7_000, 23_000, 173)) + [0, slide, size, -1]:
        brute = sorted(slide * j for j in range(-60, 60) if slide * j <= ts < slide * j + size)
        got = sorted(g.assign_windows(ts))
        assert got == brute, ts
        # every window holding ts is the union of the panes [start/pane, end/pane), one of them ts's
        p = int(g.pane_of(ts))
        for s in got:
            assert s // g.pane <= p < (s + size) // g.pane
    # a window closes with the pane ending at its end
    for p in range(-20, 40):
        s, e = g.window_of_last_pane(p)
        assert g.closes(p) == (s % slide == 0)
        assert e - s == size


def test_pane_merge_equals_window(oracle_mod):
    """Windows of 3 panes: oracle top-k per pane (idx + pane base), host merge == oracle on the
    window; objIDs repeat within and across panes (trajectories)."""
    from spatialflink_amd.spatialOperators import knn_merge_host

    og = oracle_mod.grid(500, *BEIJING)
    panes = []
    for s in range(5):
        x, y = oracle_mod.java_random_points(40 + s, 30_000, *BEIJING)
        obj = (np.random.default_rng(s).permutation(len(x)) % 12_000).astype(np.int64)
        panes.append((x, y, obj))
    for r, k in ((0.5, 50), (0.05, 20), (0.2, 300), (0.5, 1)):
        for first in range(3):
            win = panes[first:first + 3]
            lists, base = [], 0
            for x, y, obj in win:
                st, o, d, i = oracle_mod.knn(og, x, y, obj, QPOINT[0], QPOINT[1], r, k)
                assert st == 0
                lists.append((o, d, i + base))
                base += len(x)
            mo, md, mi = knn_merge_host(k, lists)
            X = np.concatenate([w[0] for w in win]); Y = np.concatenate([w[1] for w in win])
            O = np.concatenate([w[2] for w in win])
            st, eo, ed, ei = oracle_mod.knn(og, X, Y, O, QPOINT[0], QPOINT[1], r, k)
            np.testing.assert_array_equal(mo, eo)
            np.testing.assert_array_equal(md, ed)
            np.testing.assert_array_equal(mi, ei)


def test_plan_cache_keeps_pinned_plans(monkeypatch):
    """The operator plan LRU (spatialOperators._PlanCache) evicts only unpinned plans: a plan with
    a pipeline depth / capacity or held by a pane engine survives any number of other keys."""
    from spatialflink_amd import spatialOperators as so

    destroyed = []
    monkeypatch.setattr(so._PlanCache, "_destroy", lambda self, p: destroyed.append(p))
    c = so._PlanCache("unused", limit=2)
    c.put("a", 101)
    c.pin(101)
    for i, k in enumerate("bcdef"):
        c.put(k, 200 + i)
    assert c.get("a") == 101 and 101 not in destroyed
    assert len(c) == 2 and destroyed == [200, 201, 202, 203]  # the LRU unpinned ones go


def test_plan_cache_never_evicts_the_inserted_plan(monkeypatch):
    """With `limit` pinned plans, a new plan is the only unpinned entry: put() must keep it (the
    caller uses it next) and let the cache exceed its limit; unpinning restores the bound."""
    from spatialflink_amd import spatialOperators as so

    destroyed = []
    monkeypatch.setattr(so._PlanCache, "_destroy", lambda self, p: destroyed.append(p))
    c = so._PlanCache("unused", limit=3)
    for i, k in enumerate("abc"):
        c.put(k, 100 + i)
        c.pin(100 + i)
    c.put("d", 200)
    assert destroyed == [] and c.get("d") == 200 and len(c) == 4
    c.put("e", 201)  # "d" is now an ordinary LRU entry beyond the limit
    assert destroyed == [200] and c.get("e") == 201 and len(c) == 4
    c.unpin(100)  # released pin: the oldest unpinned entries go until the limit holds
    assert destroyed == [200, 100] and len(c) == 3
    assert c.get("e") == 201 and c.get("b") == 101 and c.get("c") == 102
