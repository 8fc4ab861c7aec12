"""Row-sharded FITC on ONE GPU: 2 and 3 shard contexts on device 0, each driven by its own
host thread, joined by the in-process communicator (gps_comm_init_local).  Every all-reduce
of the sharded path — the lower-packed B / b / scalar reduction of the forward, the LOO and
test-score sums, the four gradient reductions — runs at the same call sites with the same
element counts as under RCCL, the partials summed on the device in rank order, stream-ordered
on the calling streams like ncclAllReduce (round 5; test_gpu_rccl runs a real RCCL communicator).  The
sharded results must match the unsharded fit (K20:222-234, 270-296, 236/344/452).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from conftest import load_golden, nrel, record_floors, theta_of

pytestmark = pytest.mark.gpu

OBJS = ("nlml", "loo_crps", "loo_logs", "logdet", "quad")
_GROUP = [1000]


def _case(n, nt, m, d, seed):
    rng = np.random.default_rng(seed)
    X, Xt = rng.standard_normal((n, d)), rng.standard_normal((nt, d))
    w = rng.standard_normal(d) / np.sqrt(d)
    y = np.sin(3 * X @ w) + 0.1 * rng.standard_normal(n)
    yt = np.sin(3 * Xt @ w) + 0.1 * rng.standard_normal(nt)
    Z = X[rng.choice(n, m, replace=False)]
    th = (0.1, np.log(np.linspace(1.6, 2.4, d)), np.log(0.02))
    return X, y, Xt, yt, Z, th


def _run(gp, th, with_grad):
    r = gp.fit(theta=th)
    mu, var, sc = gp.predict(with_scores=True)
    out = {"obj": r.objectives, "mu_loo": r.mu_loo, "var_loo": r.var_loo, "mu": mu, "var": var,
           "sc": sc}
    if with_grad:
        for o in ("nlml", "loo_crps", "loo_logs"):
            _, g, objs = gp.value_and_grad(th, o)
            out["g_" + o] = g
            out["gz_" + o] = objs["grad_Z"]
    return out


def _sharded(P, X, y, Xt, yt, Z, th, with_grad, ar_chunks=None):
    import gpscore
    from gpscore.dist import shard_rows
    _GROUP[0] += 1
    key = _GROUP[0]
    n, nt = len(y), len(Xt)
    stats = (float(y.mean()), float(y.var(ddof=1)))

    def rank_job(r):
        ctx = gpscore.Context(0)
        try:
            ctx.call("gps_comm_init_local", P, r, key)
            if ar_chunks is not None:
                ctx.set_ar_chunks(ar_chunks)
            gp = gpscore.GP(ctx=ctx)
            a, b = shard_rows(n, P, r)
            ta, tb = shard_rows(nt, P, r)
            gp.set_data(X[a:b], y[a:b], kind="fitc", Z=Z, n_total=n, ytr_stats=stats)
            gp.set_test(Xt[ta:tb], yt[ta:tb], nt_total=nt)
            res = _run(gp, th, with_grad)
            ctx.call("gps_comm_destroy")
            return res
        finally:
            ctx.close()

    with ThreadPoolExecutor(max_workers=P) as ex:
        return list(ex.map(rank_job, range(P)))


def _whole(X, y, Xt, yt, Z, th, with_grad, gpu_ctx):
    import gpscore
    gp = gpscore.GP(ctx=gpu_ctx)
    gp.set_data(X, y, kind="fitc", Z=Z)
    gp.set_test(Xt, yt)
    return _run(gp, th, with_grad)


def _diffs(parts, ref):
    """relative differences of every global quantity (max over ranks) and of the
    concatenated row-sharded vectors"""
    out = {}
    for p in parts:
        for k in OBJS:
            out[k] = max(out.get(k, 0.0), abs(p["obj"][k] - ref["obj"][k]) / max(1.0, abs(ref["obj"][k])))
        for k, v in ref["sc"].items():
            out[k] = max(out.get(k, 0.0), abs(p["sc"][k] - v) / max(1.0, abs(v)))
        for k in ref:
            if k.startswith("g"):
                out[k] = max(out.get(k, 0.0), nrel(p[k], ref[k]))
    for k in ("mu_loo", "var_loo", "mu", "var"):
        out[k] = nrel(np.concatenate([p[k] for p in parts]), ref[k])
    return out


def _floor(X, y, Xt, yt, Z, th, with_grad, gpu_ctx, ref):
    """This problem's conditioning floor, measured: the unsharded fit at inputs perturbed
    by 1e-15 (relative; two draws) moves every output by this much.  A shard split only
    reorders sums, so it must stay within a small multiple of it."""
    fl = {}
    for seed in (1, 2):
        rng = np.random.default_rng(seed)
        Xp = X * (1 + 1e-15 * rng.standard_normal(X.shape))
        Zp = Z * (1 + 1e-15 * rng.standard_normal(Z.shape))
        for k, v in _diffs([_whole(Xp, y, Xt, yt, Zp, th, with_grad, gpu_ctx)], ref).items():
            fl[k] = max(fl.get(k, 0.0), v)
    return fl


def _compare(parts, ref, floor, cap, test, factor=30.0, abs_min=1e-13, grad_cap=None):
    d = _diffs(parts, ref)
    # absolute ceilings: test_gpu_parity.fitc_cap for the forward outputs, fitc_grad_cap (two
    # solves deep) for the θ- and Z-gradients — neither the error nor the floor may exceed it
    gcap = 2.0 * cap if grad_cap is None else grad_cap
    caps = {k: (gcap if k.startswith("g") else cap) + abs_min for k in d}
    record_floors(test, d, floor, caps)
    for k, v in sorted(d.items()):
        print(f"{k:16s} sharded {v:.2e}  floor {floor[k]:.2e}  cap {caps[k]:.2e}")
    bad = {k: (v, floor[k]) for k, v in d.items() if v > factor * floor[k] + abs_min}
    assert not bad, bad
    over = {k: (v, floor[k], caps[k]) for k, v in d.items() if max(v, floor[k]) > caps[k]}
    assert not over, over


@pytest.mark.parametrize("P", [2, 3])
def test_fitc_shards_match_unsharded(gpu_ctx, P):
    """n = 6001 (ragged shards), m = 300, d = 8: forward, predict, scores and the θ / Z
    gradients of all three objectives, each within 30× its measured conditioning floor."""
    X, y, Xt, yt, Z, th = _case(6001, 1501, 300, 8, 41)
    ref = _whole(X, y, Xt, yt, Z, th, True, gpu_ctx)
    parts = _sharded(P, X, y, Xt, yt, Z, th, True)
    from test_gpu_parity import fitc_cap
    _compare(parts, ref, _floor(X, y, Xt, yt, Z, th, True, gpu_ctx, ref), fitc_cap(Z, th),
             f"fitc_shards_P{P}")


def test_fitc_shards_large_m(gpu_ctx):
    """m = 2700 (22 tiles: the m×m factorisations recurse once, so the q and r row-norm passes
    each have a pre-pass on a second stream inside the captured factorisation, and the fit
    forms the test-side row norms), 2 shards, forward + predict: within 30× the floor."""
    X, y, Xt, yt, Z, th = _case(7001, 1201, 2700, 16, 44)  # d = 16: cond(K̃mm) ~3e3
    ref = _whole(X, y, Xt, yt, Z, th, False, gpu_ctx)
    parts = _sharded(2, X, y, Xt, yt, Z, th, False)
    from test_gpu_parity import fitc_cap
    _compare(parts, ref, _floor(X, y, Xt, yt, Z, th, False, gpu_ctx, ref), fitc_cap(Z, th),
             "fitc_shards_large_m")


def test_c5_sharded_p8(gpu_ctx):
    """BASELINE.json configs[4] in its stated form: C5 (FITC n = 200 000, m = 4000, d = 16,
    n* = 10 000, the bench's own inputs) with the rows split 8 ways — 8 shard contexts on device 0
    joined by the in-process communicator, B's all-reduce in 4 row blocks (the default) — against
    the unsharded N = 1 unit: every objective, the concatenated LOO / predictive vectors and the
    global test scores within 30× the measured floor and under fitc_cap (K20:222-234, 270-296)."""
    from test_gpu_parity import _bench_inputs, fitc_cap
    X, y, Xt, yt, Z, th = _bench_inputs("C5")
    ref = _whole(X, y, Xt, yt, Z, th, False, gpu_ctx)
    parts = _sharded(8, X, y, Xt, yt, Z, th, False)
    assert sum(len(p["mu_loo"]) for p in parts) == len(y)
    assert sum(len(p["mu"]) for p in parts) == len(yt)
    _compare(parts, ref, _floor(X, y, Xt, yt, Z, th, False, gpu_ctx, ref), fitc_cap(Z, th),
             "c5_sharded_p8")


def test_fitc_shards_golden(gpu_ctx):
    """The reference-pinned golden case, 3 shards: same objectives as the dense reference."""
    g = load_golden("fitc_n2000_m200_rows")
    th, _ = theta_of(g)
    parts = _sharded(3, g["X"], g["y"], g["Xt"], g["yt"], g["Z"], th, False)
    for p in parts:
        for k in ("nlml", "loo_crps", "loo_logs"):
            assert abs(p["obj"][k] - float(g[k])) <= 1e-8 * max(1.0, abs(float(g[k]))), k
    assert nrel(np.concatenate([p["mu_loo"] for p in parts]), g["loo_mu"]) < 1e-8
    assert nrel(np.concatenate([p["mu"] for p in parts]), g["pred_mu"]) < 1e-8


def test_fitc_shards_empty_test_shard(gpu_ctx):
    """nt_total = 2 over 3 ranks leaves one rank without test rows; its zero score partials
    still join the all-reduce and the global scores are those of the unsharded predict."""
    X, y, Xt, yt, Z, th = _case(900, 2, 60, 4, 43)
    ref = _whole(X, y, Xt, yt, Z, th, False, gpu_ctx)
    parts = _sharded(3, X, y, Xt, yt, Z, th, False)
    from test_gpu_parity import fitc_cap
    _compare(parts, ref, _floor(X, y, Xt, yt, Z, th, False, gpu_ctx, ref), fitc_cap(Z, th),
             "fitc_shards_empty_test")


def _blockloo_sharded(P, X, y, Z, th, nfold, objective, rows):
    import gpscore
    _GROUP[0] += 1
    key = _GROUP[0]
    n = len(y)
    stats = (float(y.mean()), float(y.var(ddof=1)))

    def rank_job(r):
        ctx = gpscore.Context(0)
        try:
            ctx.call("gps_comm_init_local", P, r, key)
            gp = gpscore.GP(ctx=ctx)
            a, b = rows(n, nfold, P, r)
            gp.set_data(X[a:b], y[a:b], kind="fitc", Z=Z, n_total=n, ytr_stats=stats)
            try:
                return gp.block_loo(th, objective, nfold=nfold, grad=True)
            except gpscore.GpsError as e:
                return e
            finally:
                ctx.call("gps_comm_destroy")
        finally:
            ctx.close()

    with ThreadPoolExecutor(max_workers=P) as ex:
        return list(ex.map(rank_job, range(P)))


def _blockloo_check(gpu_ctx, X, y, Z, th, nfold, objective, parts, tag):
    """every rank's (value, folds, grad, grad_Z) against the unsharded block-LOO within 30× the
    measured conditioning floor and under the absolute caps"""
    import gpscore
    gp = gpscore.GP(ctx=gpu_ctx)
    gp.set_data(X, y, kind="fitc", Z=Z)
    v0, g0, f0, gz0 = gp.block_loo(th, objective, nfold=nfold, grad=True)

    def diffs(results):
        e = {}
        for res in results:
            assert not isinstance(res, Exception), res
            v, g, f, gz = res
            e["value"] = max(e.get("value", 0.0), abs(v - v0) / abs(v0))
            e["folds"] = max(e.get("folds", 0.0), nrel(f, f0))
            e["grad"] = max(e.get("grad", 0.0), nrel(g, g0))
            e["grad_Z"] = max(e.get("grad_Z", 0.0), nrel(gz, gz0))
        return e
    errs = diffs(parts)
    # this problem's conditioning floor, measured as in _floor: the unsharded objective at
    # inputs perturbed by 1e-15 (relative, two draws)
    floor = {}
    for seed in (1, 2):
        rng = np.random.default_rng(seed)
        gp.set_data(X * (1 + 1e-15 * rng.standard_normal(X.shape)), y, kind="fitc",
                    Z=Z * (1 + 1e-15 * rng.standard_normal(Z.shape)))
        for k, v in diffs([gp.block_loo(th, objective, nfold=nfold, grad=True)]).items():
            floor[k] = max(floor.get(k, 0.0), v)
    from test_gpu_parity import fitc_cap, fitc_grad_cap
    cap, gcap = fitc_cap(Z, th), fitc_grad_cap(Z, th, depth=4)  # block-LOO: 4 solves deep
    caps = {k: (gcap if k.startswith("grad") else cap) + 1e-13 for k in errs}
    record_floors(tag, errs, floor, caps)
    print(errs, floor, caps)
    bad = {k: (v, floor[k]) for k, v in errs.items() if v > 30.0 * floor[k] + 1e-13}
    assert not bad, bad
    # absolute ceilings on the values (fitc_cap) and the θ- / Z-gradients (fitc_grad_cap)
    over = {k: (errs[k], floor[k], caps[k]) for k in errs if max(errs[k], floor[k]) > caps[k]}
    assert not over, over


@pytest.mark.parametrize("P,nfold,objective", [(2, 4, "kc"), (3, 6, "dss"), (4, 4, "kc")])
def test_fitc_blockloo_shards(gpu_ctx, P, nfold, objective):
    """FITC block-LOO (K20:523-587 DSS, K20:655-720 KC) with the rows sharded on fold
    boundaries (dist.fold_shard_rows): every rank returns the unsharded value, all fold values,
    and the θ- and Z-gradients (a shard split only reorders the n-sums)."""
    from gpscore.dist import fold_shard_rows
    X, y, _, _, Z, th = _case(4000, 10, 40, 4, 45 + P)
    parts = _blockloo_sharded(P, X, y, Z, th, nfold, objective,
                              lambda n, k, p, r: fold_shard_rows(n, k, p, r))
    _blockloo_check(gpu_ctx, X, y, Z, th, nfold, objective, parts,
                    f"fitc_blockloo_shards_P{P}_{objective}")


def test_fitc_blockloo_refuses_straddling_folds(gpu_ctx):
    """Shards that cut a fold (contiguous row shards of 4001 rows over 2 ranks, 4 folds): every
    rank reports the error — none is left waiting in an all-reduce."""
    import gpscore
    from gpscore.dist import shard_rows
    X, y, _, _, Z, th = _case(4001, 10, 30, 3, 44)
    parts = _blockloo_sharded(2, X, y, Z, th, 4, "kc",
                              lambda n, k, p, r: shard_rows(n, p, r))
    assert all(isinstance(r, gpscore.GpsError) for r in parts), parts
    assert all("straddles" in str(r) for r in parts), parts


def test_local_group_reinit_and_duplicate_rank(gpu_ctx):
    """an aborted in-process group is never rejoined — re-initialising the same key
    after a member left builds a fresh group whose all-reduces work; a second live context
    cannot take a rank another context already holds; a rank of the aborted group fails at once
    instead of waiting."""
    import gpscore
    X, y, Xt, yt, Z, th = _case(1200, 40, 50, 3, 45)
    ref = _whole(X, y, Xt, yt, Z, th, False, gpu_ctx)
    key = 777001
    c0, c1, c2 = gpscore.Context(0), gpscore.Context(0), gpscore.Context(0)
    try:
        c0.call("gps_comm_init_local", 2, 0, key)
        with pytest.raises(gpscore.GpsError, match="already holds this rank"):
            c2.call("gps_comm_init_local", 2, 0, key)
        c1.call("gps_comm_init_local", 2, 1, key)
        c1.call("gps_comm_destroy")  # member leaves: the group is aborted
        gp0 = gpscore.GP(ctx=c0)
        gp0.set_data(X[:600], y[:600], kind="fitc", Z=Z, n_total=1200,
                     ytr_stats=(float(y.mean()), float(y.var(ddof=1))))
        with pytest.raises(gpscore.GpsError, match="left the group"):
            gp0.fit(theta=th)
        # both ranks re-join the same key: a fresh group, the sharded fit matches the whole
        from gpscore.dist import shard_rows
        stats = (float(y.mean()), float(y.var(ddof=1)))

        def job(r):
            c = (c0, c1)[r]
            c.call("gps_comm_init_local", 2, r, key)
            gp = gpscore.GP(ctx=c)
            a, b = shard_rows(len(y), 2, r)
            gp.set_data(X[a:b], y[a:b], kind="fitc", Z=Z, n_total=len(y), ytr_stats=stats)
            return gp.fit(theta=th).objectives

        with ThreadPoolExecutor(max_workers=2) as ex:
            objs = list(ex.map(job, range(2)))
        for o in objs:
            for k in OBJS:
                assert abs(o[k] - ref["obj"][k]) <= 1e-9 * max(1.0, abs(ref["obj"][k])), k
    finally:
        for c in (c0, c1, c2):
            c.close()


def test_local_group_late_joiner(gpu_ctx):
    """the reduction path of an in-process group (device sums when every member is on
    one device, host sums otherwise) is read only once all ranks have joined — a rank that
    reaches its first all-reduce before a late member has joined waits for it (bounded) instead
    of fixing the path on a partial membership.  Rank 1 joins 1.5 s after rank 0 starts its fit:
    both ranks return the bits of the same two shards joined on time, and the whole fit's
    objectives within the shard tests' rounding."""
    import time

    import gpscore
    from gpscore.dist import shard_rows
    X, y, Xt, yt, Z, th = _case(1200, 40, 50, 3, 45)
    ref = _whole(X, y, Xt, yt, Z, th, False, gpu_ctx)
    stats = (float(y.mean()), float(y.var(ddof=1)))

    def sharded(delay):
        _GROUP[0] += 1
        key = _GROUP[0]

        def job(r):
            ctx = gpscore.Context(0)
            try:
                if r == 1:
                    time.sleep(delay)
                ctx.call("gps_comm_init_local", 2, r, key)
                gp = gpscore.GP(ctx=ctx)
                a, b = shard_rows(len(y), 2, r)
                gp.set_data(X[a:b], y[a:b], kind="fitc", Z=Z, n_total=len(y), ytr_stats=stats)
                out = gp.fit(theta=th).objectives
                ctx.call("gps_comm_destroy")
                return out
            finally:
                ctx.close()

        with ThreadPoolExecutor(max_workers=2) as ex:
            return list(ex.map(job, range(2)))

    late, on_time = sharded(1.5), sharded(0.0)
    for o, q in zip(late, on_time):
        assert o == q
        for k in OBJS:
            assert abs(o[k] - ref["obj"][k]) <= 1e-9 * max(1.0, abs(ref["obj"][k])), k


def test_fitc_shards_chunked_allreduce_bitwise(gpu_ctx):
    """GPS_OPT_AR_CHUNKS: B's exchange in row blocks, each all-reduced on the comm stream while
    the next block's SYRK runs, gives the same bits as one all-reduce after the whole
    SYRK — the slab values do not depend on the row blocks, and the packed sum is the same sum
    in the same order — for the forward objectives, the LOO and predictive vectors and scores."""
    X, y, Xt, yt, Z, th = _case(5000, 700, 700, 6, 47)  # m_pad = 768: 6 tile rows
    runs = {c: _sharded(2, X, y, Xt, yt, Z, th, False, ar_chunks=c) for c in (1, 4, 6)}
    base = runs[1]
    for c in (4, 6):
        for pa, pb in zip(runs[c], base):
            assert pa["obj"] == pb["obj"], c
            assert pa["sc"] == pb["sc"], c
            for k in ("mu_loo", "var_loo", "mu", "var"):
                assert np.array_equal(pa[k], pb[k]), (c, k)
