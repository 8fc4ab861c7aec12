"""The factorisation graph cache (api.hip potrf_inv): a captured launch sequence bakes in device
addresses, so no graph may outlive a buffer it uses.  Buffers that
grow drop the graphs that use them before the free; past the cache capacity the least recently used
exec is destroyed; in both cases later fits — replays, recaptures, and the shapes the test started
with — must give the same bits as the first time, with no dependency-wait timeout and no
"incomplete queue" report from the persistent factorisation.  Reference: the GD loops' repeated
fits at a fixed n (KF:237-260) and the compat calls at varying n (KF:25-29)."""
import numpy as np
import pytest

from conftest import load_golden, theta_of

pytestmark = pytest.mark.gpu


def _data(n, d=4, seed=0):
    rng = np.random.default_rng(seed + n)
    X = rng.standard_normal((n, d))
    return X, np.sin(X.sum(1)) + 0.1 * rng.standard_normal(n)


def _fit(gp, n, th):
    X, y = _data(n)
    r = gp.fit(X, y, th)
    return dict(r.objectives), r.mu_loo.copy(), r.var_loo.copy()


def _same(a, b):
    return a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])


def test_graph_cache_grow_evict_and_return():
    import gpscore
    ctx = gpscore.Context(0)
    try:
        gp = gpscore.GP(ctx=ctx)
        th = (0.0, 0.0, np.log(0.02))
        first_shapes = [300, 700, 1500]  # ascending: every fit grows A / Linv / W / vectors
        first = {n: _fit(gp, n, th) for n in first_shapes}
        s = ctx.stats()
        assert s["graph_dropped"] >= 1, s  # the growth freed buffers that earlier graphs used
        # buffers at their largest, then more distinct padded sizes than the cache holds: the
        # least recently used execs are destroyed while their buffers are alive
        cap = s["graph_cap"]
        sizes = [128 * k + 37 for k in range(cap + 8, 0, -1)]  # n_pad 128 .. 128 (cap + 8)
        ref_big = _fit(gp, sizes[0], th)
        for n in sizes[1:]:
            _fit(gp, n, th)
        s = ctx.stats()
        assert s["graph_evicted"] >= 1 and s["graphs"] <= cap, s
        assert s["graph_overflow"] == 0, s
        # back to the first shapes (evicted or still cached) and the largest one: the same bits
        for n in first_shapes:
            assert _same(_fit(gp, n, th), first[n]), n
        assert _same(_fit(gp, sizes[0], th), ref_big)
        # a replay of a cached graph is bitwise the eager launch sequence
        again = _fit(gp, 1500, th)
        ctx.set_graphs(False)
        eager = _fit(gp, 1500, th)
        ctx.set_graphs(True)
        assert _same(again, eager)
    finally:
        ctx.close()


def test_replay_after_profiled_and_other_shapes():
    """tools/diag_replay.py's sequence (the round-3 suite's "no-op replay"): a graph
    captured at one shape, then a profiled (eager) fit + predict at another, a fit at a third
    input width, then a replay — every result equals the eager fit of the same problem."""
    import gpscore
    from gpscore._lib import ptr
    g = load_golden("full_n2000_d8")
    thg, _ = theta_of(g)
    ctx = gpscore.Context(0)
    try:
        gpw = gpscore.GP(ctx=ctx)
        gpw.fit(g["X"], g["y"], thg)
        rng = np.random.default_rng(4)
        th8 = np.array([0.0, 0.3, np.log(0.01)])
        X8, Xt8, y8 = rng.standard_normal((300, 8)), rng.standard_normal((1000, 8)), rng.standard_normal(300)
        X16, y16 = rng.standard_normal((300, 16)), rng.standard_normal(300)
        out = np.zeros(8)
        ctx.call("gps_full_set_data", ptr(X8), ptr(y8), 300, 8)
        ctx.call("gps_full_set_test", ptr(Xt8), None, 1000)
        ctx.call("gps_full_set_data", ptr(X16), ptr(y16), 300, 16)
        ctx.call("gps_full_fit", 0, ptr(th8), 1, ptr(out), None, None)
        gp = gpscore.GP(ctx=ctx)
        ctx.prof(True)
        gp.fit(g["X"], g["y"], thg)
        gp.predict(g["Xt"], g["yt"])
        ctx.prof_collect()
        ctx.prof(False)
        rng = np.random.default_rng(8)
        Xa = rng.standard_normal((300, 4))
        ya = np.sin(Xa.sum(1))
        th = (0.0, 0.0, np.log(0.05))
        a = gpscore.GP(ctx=ctx)
        a.set_data(Xa, ya)
        a.set_test(Xa[:20])
        replay = a.fit(theta=th)
        ctx.set_graphs(False)
        eager = a.fit(theta=th)
        ctx.set_graphs(True)
        assert replay.objectives == eager.objectives
        assert np.array_equal(replay.mu_loo, eager.mu_loo)
    finally:
        ctx.close()
