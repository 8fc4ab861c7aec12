"""GPU k-fold block-LOO objectives (gps_full_blockloo / gps_full_blockloo_es /
gps_fitc_blockloo): DSS (KF:487-543, K20:523-587), KC (K20:655-720)
and the energy score ES (KF:607-663, ES KF:70-101), values and gradients (full GP: θ; FITC:
θ and the inducing inputs Z) against goldens composed from the reference's own dss / ES /
crps / chol_solve defs with autograd gradients (the ES draws are the reference's own
torch.randn stream, replayed), the oracle at ragged sizes and other fold counts, and finite
differences.
Tolerances (fp64): values 1e-9 relative; full-GP gradients 1e-9 normwise (ES 1e-8: C^½ by
Newton–Schulz here, by SVD in the golden); FITC as in test_gpu_fitc_grad (1e-9 for
cond(K̃mm) < 1e3, else 10× the oracle's own sensitivity to 1e-15 input perturbations);
finite differences 1e-5 relative."""
import numpy as np
import pytest

import gp_oracle as O
from conftest import golden_names, load_golden, nrel, theta_of

pytestmark = pytest.mark.gpu

BLOCK = golden_names("block_")
ES_GOLD = golden_names("blockes_")
OBJS = ("dss", "kc")


@pytest.fixture(scope="module")
def gp(gpu_ctx):
    import gpscore
    return gpscore.GP(ctx=gpu_ctx)


@pytest.mark.parametrize("name", BLOCK)
@pytest.mark.parametrize("obj", OBJS)
def test_blockloo_vs_golden(gp, name, obj):
    g = load_golden(name)
    th, _ = theta_of(g)
    ref = float(g["value_" + obj])
    if "Z" in g:
        gp.set_data(g["X"], g["y"], kind="fitc", Z=g["Z"])
        val, grad, folds, gz = gp.block_loo(th, obj, grad=True)
        Kmm, _, _ = O.fitc_shared(g["Z"], *th[:2])
        tol = 1e-9 if np.linalg.cond(Kmm) < 1e3 else 1e-6
        assert nrel(grad, g["grad_" + obj]) <= tol, (grad, g["grad_" + obj])
        assert nrel(gz, g["gradZ_" + obj]) <= tol
        assert abs(gp.block_loo(th, obj) - val) <= 1e-12 * max(1.0, abs(val))
    else:
        gp.set_data(g["X"], g["y"])
        val, grad, folds = gp.block_loo(th, obj, grad=True)
        assert nrel(grad, g["grad_" + obj]) <= 1e-9, (grad, g["grad_" + obj])
    assert abs(folds.sum() - val) <= 1e-12 * max(1.0, abs(val))
    assert abs(val - ref) <= 1e-9 * max(1.0, abs(ref)), (val, ref)


@pytest.mark.parametrize("name", ES_GOLD)
def test_es_vs_golden(gp, name):
    """ES with the reference's draws: value and the `.backward()` of KF:663."""
    g = load_golden(name)
    th, _ = theta_of(g)
    S = int(g["num_sim"])
    gp.set_data(g["X"], g["y"])
    val, grad, folds = gp.block_loo(th, "es", grad=True, num_sim=S, draws=g["draws_es"])
    ref = float(g["value_es"])
    assert abs(val - ref) <= 1e-9 * max(1.0, abs(ref)), (val, ref)
    assert nrel(grad, g["grad_es"]) <= 1e-8, (grad, g["grad_es"])
    assert abs(folds.sum() - val) <= 1e-12 * max(1.0, abs(val))
    assert abs(gp.block_loo(th, "es", num_sim=S, draws=g["draws_es"]) - val) <= 1e-12 * abs(val)


@pytest.mark.parametrize("n,d,nfold,S,beta", [(1001, 3, 4, 64, 1.0), (777, 2, 3, 300, 1.0),
                                              (2600, 8, 4, 100, 1.0), (500, 4, 4, 50, 1.5)])
def test_es_vs_oracle(gp, n, d, nfold, S, beta):
    """Unequal folds, other fold counts and draw counts, β != 1; larger folds (b = 650)."""
    from gpscore.gp import es_draws
    rng = np.random.default_rng(n + S)
    X = rng.standard_normal((n, d))
    y = np.sin(X.sum(1)) + 0.1 * rng.standard_normal(n)
    th = (0.1, np.log(np.linspace(0.8, 2.0, d)), np.log(0.05))
    draws = es_draws(n, nfold, S, rng)
    gp.set_data(X, y)
    val, grad, _ = gp.block_loo(th, "es", nfold=nfold, grad=True, num_sim=S, beta=beta, draws=draws)
    es = {"draws": draws, "S": S, "beta": beta}
    ov, og = O.fast_full_blockloo(X, y, *th, "es", nfold=nfold, want_grad=True, es=es)
    assert abs(val - ov) <= 1e-9 * max(1.0, abs(ov)), (val, ov)
    assert nrel(grad, og) <= 1e-8, (grad, og)


def test_es_finite_difference(gp):
    """n = 4096 (folds of 1024), fixed draws: directional derivative vs grad · direction."""
    from gpscore.gp import es_draws
    rng = np.random.default_rng(29)
    n, d, S = 4096, 8, 64
    X = rng.standard_normal((n, d))
    y = np.sin(X @ rng.standard_normal(d) / np.sqrt(d)) + 0.1 * rng.standard_normal(n)
    draws = es_draws(n, 4, S, rng)
    gp.set_data(X, y)
    th = np.concatenate([[0.0], np.log(np.linspace(1.2, 2.4, d)), [np.log(0.02)]])
    val, grad, _ = gp.block_loo((th[0], th[1:-1], th[-1]), "es", grad=True, num_sim=S, draws=draws)
    u = rng.standard_normal(th.size)
    u /= np.linalg.norm(u)
    h = 1e-5

    def f(t):
        return gp.block_loo((t[0], t[1:-1], t[-1]), "es", num_sim=S, draws=draws)

    fd = (f(th + h * u) - f(th - h * u)) / (2 * h)
    assert abs(fd - grad @ u) <= 1e-5 * max(abs(fd), np.linalg.norm(grad) * 1e-3), (fd, grad @ u)


def test_compat_es_dss_vs_golden(gpu_ctx):
    """compat.ES / compat.dss (KF:70-108) on one Gaussian with the reference's draws; ES with a
    general C converges the Newton–Schulz iteration on ‖I − ZY‖ (gps_energy_score)."""
    from gpscore import compat
    g = load_golden("es_single")
    b = g["C"].shape[0]
    v = compat.ES(g["m"], g["C"], b, g["y"], int(g["num_sim"]), draws=g["draws"])
    assert abs(v - float(g["es"])) <= 1e-10 * max(1.0, abs(float(g["es"]))), (v, float(g["es"]))
    dv = compat.dss(g["m"], g["C"], b, g["y"])
    assert abs(dv - float(g["dss"])) <= 1e-10 * max(1.0, abs(float(g["dss"]))), (dv, float(g["dss"]))


@pytest.mark.parametrize("tag", ["well", "ill"])
def test_compat_dss_vs_k20_golden(gpu_ctx, tag):
    """compat.dss (gps_potrs / gps_potrf on the device) against K20's own dss def (K20:106-111,
    cov_term.inverse()) and KF's (KF:103-108) from the dss_k20 golden: within the covariance's
    cond·ε, as the two reference defs differ from each other."""
    from gpscore import compat
    g = load_golden("dss_k20")
    C = g[f"{tag}_C"]
    b = C.shape[0]
    dv = compat.dss(g[f"{tag}_m"], C, b, g[f"{tag}_y"])
    tol = 1e-12 if tag == "well" else 1e-15 * np.linalg.cond(C)
    for k in ("dss_k20", "dss_kf"):
        ref = float(g[f"{tag}_{k}"])
        assert abs(dv - ref) <= tol * abs(ref), (k, dv, ref)


def test_es_sgd_train(gp):
    """The KF:663-672 SGD loop on ES through GP.train (3 steps, fresh draws per step from one
    Generator) vs the oracle replaying the same draws."""
    from gpscore.gp import es_draws
    g = load_golden("blockes_full_n64")
    th, _ = theta_of(g)
    lr, S = 0.1, 32
    theta, series = gp.train(th, "es", lr=lr, itr=3, X=g["X"], y=g["y"],
                             block_kw={"num_sim": S, "rng": np.random.default_rng(3)})
    rng = np.random.default_rng(3)
    t = np.concatenate([[th[0]], np.atleast_1d(th[1]), [th[2]]])
    for i in range(3):
        es = {"draws": es_draws(g["X"].shape[0], 4, S, rng), "S": S}
        v, gr = O.fast_full_blockloo(g["X"], g["y"], t[0], t[1:-1], t[-1], "es", want_grad=True, es=es)
        assert abs(v - series["objective"][i]) <= 1e-9 * abs(v)
        t = t - lr * gr
        assert nrel(series["theta"][i], t) <= 1e-9


@pytest.mark.parametrize("n,d,nfold,iso", [(1001, 3, 4, False), (3000, 8, 4, False),
                                           (777, 2, 3, True), (1500, 5, 7, False)])
@pytest.mark.parametrize("obj", OBJS)
def test_full_blockloo_vs_oracle(gp, n, d, nfold, iso, obj):
    """Unequal folds (n % k != 0), other fold counts, scalar and per-dimension ℓ."""
    rng = np.random.default_rng(n + d + nfold)
    X = rng.standard_normal((n, d))
    y = np.sin(X.sum(1)) + 0.1 * rng.standard_normal(n)
    th = (0.1, np.log(1.3) if iso else np.log(np.linspace(0.8, 2.0, d)), np.log(0.05))
    gp.set_data(X, y)
    val, grad, _ = gp.block_loo(th, obj, nfold=nfold, grad=True)
    ov, og = O.fast_full_blockloo(X, y, *th, obj, nfold=nfold, want_grad=True)
    assert abs(val - ov) <= 1e-9 * max(1.0, abs(ov))
    assert nrel(grad, og) <= 1e-9, (grad, og)
    assert abs(gp.block_loo(th, obj, nfold=nfold) - val) <= 1e-12 * max(1.0, abs(val))


@pytest.mark.parametrize("n,m,nfold", [(2000, 150, 4), (1001, 37, 3)])
@pytest.mark.parametrize("obj", OBJS)
def test_fitc_blockloo_vs_oracle(gp, n, m, nfold, obj):
    rng = np.random.default_rng(n + m)
    d = 6
    X = rng.standard_normal((n, d))
    y = np.sin(X.sum(1)) + 0.1 * rng.standard_normal(n)
    Z = X[rng.choice(n, m, replace=False)]
    th = (0.0, np.log(np.linspace(1.0, 2.5, d)), np.log(0.05))
    gp.set_data(X, y, kind="fitc", Z=Z)
    val, grad, _, gz = gp.block_loo(th, obj, nfold=nfold, grad=True)
    ov, og, oz = O.fast_fitc_blockloo(X, y, Z, *th, obj, nfold=nfold, want_grad=True)
    assert abs(val - ov) <= 1e-9 * max(1.0, abs(ov)), (val, ov)
    # tolerance: 10× the oracle's own change under 1e-15 relative input perturbations
    r = np.random.default_rng(1)
    _, pg, pz = O.fast_fitc_blockloo(X * (1 + 1e-15 * r.standard_normal(X.shape)), y,
                                     Z * (1 + 1e-15 * r.standard_normal(Z.shape)), *th, obj,
                                     nfold=nfold, want_grad=True)
    tol = max(1e-9, 10 * max(nrel(pg, og), nrel(pz, oz)))
    assert tol < 1e-4
    assert nrel(grad, og) <= tol and nrel(gz, oz) <= tol, (tol, nrel(grad, og), nrel(gz, oz))


@pytest.mark.parametrize("obj", OBJS)
def test_fitc_blockloo_lowrank_vs_oracle(gp, obj):
    """The FITC folds in low rank (round 5: C_f = Λ_f + WWᵀ with W = K_f L_{-f}^-T never formed,
    O(b·m²) per fold) against the oracle's dense b×b fold covariance: unequal folds (n = 3001),
    values 1e-9 relative, θ- and Z-gradients within the oracle-perturbation tolerance above.  The
    dense GPU path it replaced measured 243.5 → 85.7 ms (KC) per C4 GD iteration
    (profiles/r5o_fitc_lowrank_ab.txt)."""
    rng = np.random.default_rng(77)
    n, m, d, nfold = 3001, 180, 5, 4
    X = rng.standard_normal((n, d))
    y = np.sin(X.sum(1)) + 0.1 * rng.standard_normal(n)
    Z = X[rng.choice(n, m, replace=False)]
    th = (0.1, np.log(np.linspace(1.0, 2.0, d)), np.log(0.04))
    gp.set_data(X, y, kind="fitc", Z=Z)
    val, grad, folds, gz = gp.block_loo(th, obj, nfold=nfold, grad=True)
    ov, og, oz = O.fast_fitc_blockloo(X, y, Z, *th, obj, nfold=nfold, want_grad=True)
    r = np.random.default_rng(2)
    _, pg, pz = O.fast_fitc_blockloo(X * (1 + 1e-15 * r.standard_normal(X.shape)), y,
                                     Z * (1 + 1e-15 * r.standard_normal(Z.shape)), *th, obj,
                                     nfold=nfold, want_grad=True)
    tol = max(1e-9, 10 * max(nrel(pg, og), nrel(pz, oz)))
    assert tol < 1e-4
    assert nrel(grad, og) <= tol and nrel(gz, oz) <= tol, (tol, nrel(grad, og), nrel(gz, oz))
    assert abs(val - ov) <= 1e-9 * max(1.0, abs(ov)), (val, ov)
    assert abs(folds.sum() - val) <= 1e-12 * max(1.0, abs(val))


@pytest.mark.parametrize("obj", OBJS)
def test_fitc_blockloo_finite_difference(gp, obj):
    """n = 6000, m = 200: directional derivative of the GPU objective along a random direction
    in (θ, Z) vs grad · direction."""
    rng = np.random.default_rng(23)
    n, m, d = 6000, 200, 6
    X = rng.standard_normal((n, d))
    y = np.sin(X @ rng.standard_normal(d) / np.sqrt(d)) + 0.1 * rng.standard_normal(n)
    Z = X[rng.choice(n, m, replace=False)]
    th = np.concatenate([[0.0], np.log(np.linspace(1.2, 2.4, d)), [np.log(0.02)]])
    gp.set_data(X, y, kind="fitc", Z=Z)
    val, grad, _, gz = gp.block_loo((th[0], th[1:-1], th[-1]), obj, grad=True)
    u = rng.standard_normal(th.size)
    uz = rng.standard_normal(Z.shape)
    nu = np.sqrt(np.sum(u * u) + np.sum(uz * uz))
    u, uz = u / nu, uz / nu
    h = 1e-4

    def f(t, z):
        gp.set_inducing(z)
        return gp.block_loo((t[0], t[1:-1], t[-1]), obj)

    fd = (f(th + h * u, Z + h * uz) - f(th - h * u, Z - h * uz)) / (2 * h)
    an = grad @ u + np.sum(gz * uz)
    scale = max(abs(fd), 1e-3 * np.sqrt(np.sum(grad ** 2) + np.sum(gz ** 2)))
    # the difference quotient's rounding floor, measured: the objective's movement under a
    # 1e-15 relative perturbation of Z (cond(K̃mm) at m = 200 makes it ~1e-12-1e-11 relative,
    # and it moves with the GEMM's summation order), divided by h, with a 10× margin
    pert = [abs(f(th, Z * (1 + 1e-15 * rng.standard_normal(Z.shape))) - val) for _ in range(2)]
    floor = 10 * max(pert + [1e-13 * abs(val)]) / h
    assert abs(fd - an) <= 1e-5 * scale + floor, (fd, an, floor)


def test_fitc_blockloo_sgd_train(gp):
    """Three steps of the K20:666-726 KC loop (θ and inducing_x) through GP.train vs the oracle."""
    g = load_golden("block_fitc_n500_m20")
    th, _ = theta_of(g)
    lr = 0.1
    theta, series = gp.train(th, "kc", lr=lr, itr=3, X=g["X"], y=g["y"], Z0=g["Z"])
    t = np.concatenate([[th[0]], np.atleast_1d(th[1]), [th[2]]])
    Z = g["Z"].copy()
    for i in range(3):
        v, gr, gz = O.fast_fitc_blockloo(g["X"], g["y"], Z, t[0], t[1:-1], t[-1], "kc",
                                         want_grad=True)
        assert abs(v - series["objective"][i]) <= 1e-9 * abs(v)
        t = t - lr * gr
        Z = Z - lr * gz
        assert nrel(series["theta"][i], t) <= 1e-9
    assert nrel(series["Z"], Z) <= 1e-9


@pytest.mark.parametrize("obj", OBJS)
def test_full_blockloo_finite_difference(gp, obj):
    """n = 4096: directional derivative of the GPU objective vs grad · direction."""
    rng = np.random.default_rng(17)
    n, d = 4096, 8
    X = rng.standard_normal((n, d))
    y = np.sin(X @ rng.standard_normal(d) / np.sqrt(d)) + 0.1 * rng.standard_normal(n)
    gp.set_data(X, y)
    th = np.concatenate([[0.0], np.log(np.linspace(1.2, 2.4, d)), [np.log(0.02)]])
    val, grad, _ = gp.block_loo((th[0], th[1:-1], th[-1]), obj, grad=True)
    u = rng.standard_normal(th.size)
    u /= np.linalg.norm(u)
    h = 1e-5

    def f(t):
        return gp.block_loo((t[0], t[1:-1], t[-1]), obj)

    fd = (f(th + h * u) - f(th - h * u)) / (2 * h)
    assert abs(fd - grad @ u) <= 1e-5 * max(abs(fd), np.linalg.norm(grad) * 1e-3), (fd, grad @ u)


def test_blockloo_sgd_train(gp):
    """The KF:543-550 SGD loop on the DSS objective through GP.train (3 steps) vs the oracle."""
    g = load_golden("block_full_n64")
    th, _ = theta_of(g)
    lr = 1e-3
    theta, series = gp.train(th, "dss", lr=lr, itr=3, X=g["X"], y=g["y"])
    t = np.concatenate([[th[0]], np.atleast_1d(th[1]), [th[2]]])
    for i in range(3):
        v, gr = O.fast_full_blockloo(g["X"], g["y"], t[0], t[1:-1], t[-1], "dss", want_grad=True)
        assert abs(v - series["objective"][i]) <= 1e-9 * abs(v)
        t = t - lr * gr
        assert nrel(series["theta"][i], t) <= 1e-9
