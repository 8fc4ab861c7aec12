"""The replicate harness (gpscore.experiment) on the GPU against the
same loop driven by the oracle: SGD on the oracle's gradients from the same start (and the
same ES draws), then the stale-σ² predictor and the score bundle (KF:267-299).
Tolerance: 1e-8 relative on every metric (a few SGD steps at the scripts' learning rates)."""
import numpy as np
import pytest

import gp_oracle as O
from conftest import nrel

pytestmark = pytest.mark.gpu

ITR = 3


@pytest.fixture(scope="module")
def data():
    from gpscore import experiment as E
    sheets = E.synthetic_sheets(4, n_pool=2000, n_test=300, d=8)
    return E.replicate(sheets, j=1, n_pool=2000)


def _check(res, ref):
    for k, rk in (("mse", "test_mse"), ("smse", "test_smse"), ("logs", "test_logs"),
                  ("crps", "test_crps"), ("msll", "test_msll")):
        assert abs(res[k] - ref[rk]) <= 1e-8 * max(1.0, abs(ref[rk])), (k, res[k], ref[rk])
    assert res["cover"] == pytest.approx(ref["test_cover"], abs=1e-12)


@pytest.mark.parametrize("name", ["crps", "nlml", "logs", "dss", "es"])
def test_full_method_matches_oracle_loop(gpu_ctx, data, name):
    import gpscore
    from gpscore import experiment as E
    from gpscore.gp import es_draws
    meth = E.KF_METHODS[name]
    gp = gpscore.GP(ctx=gpu_ctx)
    res = E.run_method(gp, data, meth, np.random.default_rng(11), itr=ITR, num_sim=20)
    rng = np.random.default_rng(11)
    k0, l0, s0 = E.initial_theta(meth, 8, rng)
    t = np.concatenate([[k0], np.atleast_1d(l0), [s0]])
    X, y = data["train_x"], data["train_y"]
    noise = t[-1]
    for _ in range(ITR):
        noise = t[-1]  # the forward pass's σ² (read by the predictive: stale by one step)
        if meth.objective in ("dss", "es"):
            es = ({"draws": es_draws(X.shape[0], 4, 20, rng), "S": 20}
                  if meth.objective == "es" else None)
            _, g = O.fast_full_blockloo(X, y, t[0], t[1:-1], t[-1], meth.objective,
                                        want_grad=True, es=es)
        else:
            _, g = O.fast_full_grad(X, y, t[0], t[1:-1], t[-1], meth.objective)
        t = t - meth.lr * g
    assert nrel(np.concatenate([[res["theta"][0]], np.atleast_1d(res["theta"][1]),
                                [res["theta"][2]]]), t) <= 1e-9
    ref = O.fast_full(X, y, data["test_x"], data["test_y"], t[0], t[1:-1], noise)
    _check(res, ref)


@pytest.mark.parametrize("name", ["nlml", "kc"])
def test_fitc_method_matches_oracle_loop(gpu_ctx, data, name):
    import gpscore
    from gpscore import experiment as E
    meth = E.K20_METHODS[name]
    gp = gpscore.GP(ctx=gpu_ctx)
    res = E.run_method(gp, data, meth, np.random.default_rng(5), kind="fitc", itr=ITR)
    rng = np.random.default_rng(5)
    k0, l0, s0 = E.initial_theta(meth, 8, rng)
    Z = rng.random((20, 8))
    t = np.concatenate([[k0], np.atleast_1d(l0), [s0]])
    X, y = data["train_x"], data["train_y"]
    noise = t[-1]
    for _ in range(ITR):
        noise = t[-1]
        if meth.objective == "kc":
            _, g, gz = O.fast_fitc_blockloo(X, y, Z, t[0], t[1:-1], t[-1], "kc", want_grad=True)
        else:
            _, g, gz = O.fast_fitc_grad(X, y, Z, t[0], t[1:-1], t[-1], meth.objective)
        t = t - meth.lr * g
        Z = Z - meth.lr_z * gz
    assert nrel(res["Z"], Z) <= 1e-9
    ref = O.fast_fitc(X, y, data["test_x"], data["test_y"], Z, t[0], t[1:-1], noise)
    _check(res, ref)
