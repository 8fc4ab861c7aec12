"""GPU analytic FITC gradients (gps_fitc_grad) w.r.t. theta and the inducing inputs Z,
against the reference's own autograd `.backward()` through its dense n×n FITC bodies
(K20:236 LOO-CRPS, K20:344 NLML, K20:452 LOO-LogS) captured in the goldens, the
oracle's O(n·m²) restatement (oracle.fast_fitc_grad) at ragged sizes, finite
differences at a size the dense reference cannot reach, and the SGD loop that also
moves inducing_x (K20:238-247).  Runs on the GPU box.

Tolerances (fp64): GPU vs oracle normwise 1e-9; vs the autograd goldens 1e-9 when
K̃mm is well conditioned, 1e-6 for the cond(K̃mm) ≈ 5e3 uniform-Z cases (the dense
reference's LU solves limit agreement there; see test_oracle_golden); finite
differences 1e-5 relative (central, h = 1e-5)."""
import numpy as np
import pytest

import gp_oracle as O
from conftest import golden_names, load_golden, nrel, theta_of

pytestmark = pytest.mark.gpu

FITC_GRAD = [n for n in golden_names("fitc_") if "grad_nlml" in load_golden(n)]
OBJS = ("nlml", "loo_crps", "loo_logs")


@pytest.fixture(scope="module")
def gp(gpu_ctx):
    import gpscore
    return gpscore.GP(ctx=gpu_ctx)


@pytest.mark.parametrize("name", FITC_GRAD)
@pytest.mark.parametrize("obj", OBJS)
def test_fitc_grad_vs_autograd_golden(gp, name, obj):
    g = load_golden(name)
    th, _ = theta_of(g)
    val, grad, objs = gp.value_and_grad(th, obj, X=g["X"], y=g["y"], Z=g["Z"])
    Kmm, _, _ = O.fitc_shared(g["Z"], *th[:2])
    tol = 1e-9 if np.linalg.cond(Kmm) < 1e3 else 1e-6
    ref = float(g["value_" + obj])
    assert abs(val - ref) <= 1e-9 * max(1.0, abs(ref))
    assert nrel(grad, g["grad_" + obj]) <= tol, (grad, g["grad_" + obj])
    assert nrel(objs["grad_Z"], g["gradZ_" + obj]) <= tol
    # and against the oracle's restatement at the same inputs
    ov, og, oz = O.fast_fitc_grad(g["X"], g["y"], g["Z"], *th, obj)
    assert nrel(grad, og) <= tol and nrel(objs["grad_Z"], oz) <= tol


def _shape_case(n, m, d, iso, well_conditioned=True):
    rng = np.random.default_rng(n + m + d)
    X = rng.standard_normal((n, d))
    y = np.sin(X.sum(1)) + 0.1 * rng.standard_normal(n)
    if well_conditioned:
        Z = (np.linspace(-2, 2, m)[:, None] if d == 1 else X[rng.choice(n, m, replace=False)])
        ell = (np.log(0.8 * np.sqrt(d)) if iso
               else np.log(np.linspace(0.5, 1.2, d) * np.sqrt(d) / 2))
    else:  # near-duplicate inducing points and long length-scales: cond(K̃mm) ~ 1e4
        Z = X[rng.choice(n, m, replace=False)] + 0.05 * rng.standard_normal((m, d))
        ell = np.log(np.linspace(1.0, 3.0, d))
    return X, y, Z, (0.1, ell, np.log(0.05))


@pytest.mark.parametrize("n,m,d,iso", [(1000, 37, 3, False), (3000, 300, 8, False),
                                       (700, 129, 20, False), (2000, 100, 16, True),
                                       (257, 5, 1, True)])
@pytest.mark.parametrize("obj", OBJS)
def test_fitc_grad_vs_oracle_shapes(gp, n, m, d, iso, obj):
    """Ragged n, m (not multiples of 128), d = 1 / 3 / 8 / 16 / 20 (generic-d kernel),
    scalar and per-dimension ℓ; well-conditioned K̃mm (cond <= 4e3), tolerance 1e-9."""
    X, y, Z, th = _shape_case(n, m, d, iso)
    val, grad, objs = gp.value_and_grad(th, obj, X=X, y=y, Z=Z)
    ov, og, oz = O.fast_fitc_grad(X, y, Z, *th, obj)
    assert abs(val - ov) <= 1e-9 * max(1.0, abs(ov))
    assert nrel(grad, og) <= 1e-9, (grad, og)
    assert nrel(objs["grad_Z"], oz) <= 1e-9


@pytest.mark.parametrize("obj", OBJS)
def test_fitc_grad_ill_conditioned(gp, obj):
    """cond(K̃mm) ≈ 1.8e4 (near-duplicate inducing points).  The whitened gradient
    moves by ~3e-9 under 1e-15 relative input perturbations (the round-3 explicit-inverse form:
    up to 1.2e-4); the GPU must agree with the oracle, and the GPU's own perturbation floor must
    stay, under the absolute gradient ceiling fitc_grad_cap = 100·κ·ε."""
    from conftest import record_floors
    from test_gpu_parity import fitc_grad_cap
    X, y, Z, th = _shape_case(1000, 37, 3, False, well_conditioned=False)
    val, grad, objs = gp.value_and_grad(th, obj, X=X, y=y, Z=Z)
    ov, og, oz = O.fast_fitc_grad(X, y, Z, *th, obj)
    r = np.random.default_rng(1)
    Xp, Zp = X * (1 + 1e-15 * r.standard_normal(X.shape)), Z * (1 + 1e-15 * r.standard_normal(Z.shape))
    _, pg, pobjs = gp.value_and_grad(th, obj, X=Xp, y=y, Z=Zp)
    cap = fitc_grad_cap(Z, th)
    err = {"grad": nrel(grad, og), "grad_Z": nrel(objs["grad_Z"], oz)}
    floor = {"grad": nrel(pg, grad), "grad_Z": nrel(pobjs["grad_Z"], objs["grad_Z"])}
    record_floors(f"fitc_grad_ill_{obj}", err, floor, {k: cap for k in err})
    for k in err:
        assert max(err[k], floor[k]) <= cap, (k, err[k], floor[k], cap)


@pytest.mark.parametrize("obj", OBJS)
def test_fitc_grad_finite_difference(gp, obj):
    """n = 20000, m = 400: directional derivative of the GPU objective along a random
    direction in (theta, Z) vs grad · direction."""
    rng = np.random.default_rng(11)
    n, m, d = 20000, 400, 8
    X = rng.standard_normal((n, d))
    y = np.sin(X @ rng.standard_normal(d) / np.sqrt(d)) + 0.1 * rng.standard_normal(n)
    Z = X[rng.choice(n, m, replace=False)]
    th = np.concatenate([[0.0], np.log(np.linspace(1.2, 2.4, d)), [np.log(0.02)]])
    val, grad, objs = gp.value_and_grad((th[0], th[1:-1], th[-1]), obj, X=X, y=y, Z=Z)
    u = rng.standard_normal(th.size)
    uz = rng.standard_normal(Z.shape)
    nu = np.sqrt(np.sum(u * u) + np.sum(uz * uz))
    u, uz = u / nu, uz / nu
    h = 1e-5

    def f(t, z):
        gp.set_inducing(z)
        return gp.fit(theta=(t[0], t[1:-1], t[-1]), kind="fitc", return_loo=False).objectives[obj]

    fd = (f(th + h * u, Z + h * uz) - f(th - h * u, Z - h * uz)) / (2 * h)
    an = grad @ u + np.sum(objs["grad_Z"] * uz)
    scale = max(abs(fd), 1e-3 * np.sqrt(np.sum(grad ** 2) + np.sum(objs["grad_Z"] ** 2)))
    assert abs(fd - an) <= 1e-5 * scale, (fd, an)


def test_fitc_sgd_train_matches_oracle(gp):
    """Three SGD steps of the K20:238-247 update (theta and inducing_x) vs the oracle."""
    g = load_golden("fitc_n500_m20_rows")
    th, _ = theta_of(g)
    lr, lr_z = 0.5, 0.2
    theta, series = gp.train(th, "loo_crps", lr=lr, itr=3, X=g["X"], y=g["y"], Z0=g["Z"],
                             lr_z=lr_z)
    t = np.concatenate([[th[0]], np.atleast_1d(th[1]), [th[2]]])
    Z = g["Z"].copy()
    for i in range(3):
        v, gr, gz = O.fast_fitc_grad(g["X"], g["y"], Z, t[0], t[1:-1], t[-1], "loo_crps")
        assert abs(v - series["objective"][i]) <= 1e-9 * abs(v)
        t = t - lr * gr
        Z = Z - lr_z * gz
        assert nrel(series["theta"][i], t) <= 1e-9
    assert nrel(series["Z"], Z) <= 1e-9


def test_fitc_grad_single_rank_comm_matches(gpu_ctx):
    """The sharded code path (the four all-reduces inside gps_fitc_grad) on a 1-rank RCCL
    communicator gives the communicator-free gradient."""
    import ctypes
    import gpscore
    g = load_golden("fitc_n500_m20_rows")
    th, _ = theta_of(g)
    va, ga, oa = gpscore.GP(ctx=gpu_ctx).value_and_grad(th, "loo_logs", X=g["X"], y=g["y"],
                                                        Z=g["Z"])
    ctx = gpscore.Context(0)
    lib = gpscore.load()
    buf = ctypes.create_string_buffer(128)
    assert lib.gps_comm_unique_id(buf) == 0
    ctx.call("gps_comm_init", 1, 0, buf)
    vb, gb, ob = gpscore.GP(ctx=ctx).value_and_grad(th, "loo_logs", X=g["X"], y=g["y"], Z=g["Z"])
    assert abs(va - vb) <= 1e-13 * abs(va)
    assert nrel(gb, ga) <= 1e-13 and nrel(ob["grad_Z"], oa["grad_Z"]) <= 1e-13
    ctx.call("gps_comm_destroy")
    ctx.close()
