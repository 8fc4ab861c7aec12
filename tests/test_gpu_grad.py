"""GPU analytic gradients (gps_full_grad) against the reference's own autograd
`.backward()` captured in the goldens (KF:252 / KF:339 / KF:428), the oracle's
analytic restatement at ragged sizes, a finite-difference check at a size the
oracle would be slow for, and the SGD loop (KF:254-260).  Runs on the GPU box.

Tolerances: normwise relative 1e-9 against goldens / oracle (fp64, same cond(A)·ε
argument as the forward parity); finite differences 1e-5 (central, h = 1e-5)."""
import numpy as np
import pytest

import gp_oracle as O
from conftest import golden_names, load_golden, nrel, theta_of

pytestmark = pytest.mark.gpu

GRAD = [n for n in golden_names("sd_") + golden_names("full_") if "grad_nlml" in load_golden(n)]
OBJS = ("nlml", "loo_crps", "loo_logs")


@pytest.fixture(scope="module")
def gp(gpu_ctx):
    import gpscore
    return gpscore.GP(ctx=gpu_ctx)


@pytest.mark.parametrize("name", GRAD)
@pytest.mark.parametrize("obj", OBJS)
def test_grad_vs_autograd_golden(gp, name, obj):
    g = load_golden(name)
    th, kern = theta_of(g)
    val, grad, _ = gp.value_and_grad(th, obj, X=g["X"], y=g["y"], rbf=(kern == "rbf"))
    assert abs(val - float(g[obj])) <= 1e-9 * max(1.0, abs(float(g[obj])))
    assert nrel(grad, g["grad_" + obj]) <= 1e-9, (grad, g["grad_" + obj])


@pytest.mark.parametrize("n,d,iso,rbf", [(129, 1, True, False), (1000, 3, False, False),
                                         (1500, 20, False, False), (2500, 8, False, False),
                                         (700, 2, True, True)])
@pytest.mark.parametrize("obj", OBJS)
def test_grad_vs_oracle_shapes(gp, n, d, iso, rbf, obj):
    rng = np.random.default_rng(n + d)
    X = rng.standard_normal((n, d))
    y = np.sin(X.sum(1)) + 0.1 * rng.standard_normal(n)
    ell = np.log(1.3) if iso else np.log(np.linspace(0.8, 2.5, d))
    th = (0.1, ell, np.log(0.03))
    kind = "rbf" if rbf else "ARD"
    val, grad, _ = gp.value_and_grad(th, obj, X=X, y=y, rbf=rbf)
    ov, og = O.fast_full_grad(X, y, *th, obj, kind=kind)
    assert abs(val - ov) <= 1e-9 * max(1.0, abs(ov))
    assert nrel(grad, og) <= 1e-9, (grad, og)


@pytest.mark.parametrize("obj", OBJS)
def test_grad_finite_difference(gp, obj):
    """n = 4096: directional derivative of the GPU objective vs grad · direction."""
    rng = np.random.default_rng(7)
    n, d = 4096, 8
    X = rng.standard_normal((n, d))
    y = np.sin(X @ rng.standard_normal(d) / np.sqrt(d)) + 0.1 * rng.standard_normal(n)
    gp.set_data(X, y)
    th = np.concatenate([[0.0], np.log(np.linspace(1.2, 2.4, d)), [np.log(0.02)]])
    val, grad, _ = gp.value_and_grad((th[0], th[1:-1], th[-1]), obj)
    u = rng.standard_normal(th.size)
    u /= np.linalg.norm(u)
    h = 1e-5

    def f(t):
        return gp.fit(theta=(t[0], t[1:-1], t[-1]), return_loo=False).objectives[obj]

    fd = (f(th + h * u) - f(th - h * u)) / (2 * h)
    assert abs(fd - grad @ u) <= 1e-5 * max(abs(fd), np.linalg.norm(grad) * 1e-3), (fd, grad @ u)


def test_sgd_train_matches_oracle(gp):
    """Five SGD steps (KF:254-260 update rule, lr = 1) on the GPU vs the oracle."""
    g = load_golden("full_n64_d8")
    th, _ = theta_of(g)
    theta, series = gp.train(th, "loo_crps", lr=1.0, itr=5, X=g["X"], y=g["y"])
    t = np.concatenate([[th[0]], np.atleast_1d(th[1]), [th[2]]])
    for i in range(5):
        v, gr = O.fast_full_grad(g["X"], g["y"], t[0], t[1:-1], t[-1], "loo_crps")
        assert abs(v - series["objective"][i]) <= 1e-9 * abs(v)
        t = t - gr
        assert nrel(series["theta"][i], t) <= 1e-9
    assert nrel(np.concatenate([[theta[0]], theta[1], [theta[2]]]), t) <= 1e-9
