"""GPU k-fold block-LOO objectives (gps_full_blockloo / gps_fitc_blockloo; SURVEY.md §8f
next-2): DSS (KF:487-543, K20:523-587) and KC (K20:655-720) against goldens composed from
the reference's own dss / crps / chol_solve defs (autograd gradients for the full GP),
the oracle at ragged sizes and other fold counts, and finite differences.
Tolerances (fp64): 1e-9 normwise vs goldens / oracle; finite differences 1e-5 relative."""
import numpy as np
import pytest

import gp_oracle as O
from conftest import golden_names, load_golden, nrel, theta_of

pytestmark = pytest.mark.gpu

BLOCK = golden_names("block_")
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
        val = gp.block_loo(th, obj)
    else:
        gp.set_data(g["X"], g["y"])
        val, grad, folds = gp.block_loo(th, obj, grad=True)
        assert nrel(grad, g["grad_" + obj]) <= 1e-9, (grad, g["grad_" + obj])
        assert abs(folds.sum() - val) <= 1e-12 * max(1.0, abs(val))
    assert abs(val - ref) <= 1e-9 * max(1.0, abs(ref)), (val, ref)


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
    val = gp.block_loo(th, obj, nfold=nfold)
    ov = O.fast_fitc_blockloo(X, y, Z, *th, obj, nfold=nfold)
    assert abs(val - ov) <= 1e-9 * max(1.0, abs(ov)), (val, ov)


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
