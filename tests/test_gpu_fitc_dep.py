"""GPS_OPT_FITC_DEP: the FITC row norms q_i = ‖Lm⁻¹k_i‖² and r_i = ‖Lb⁻¹k_i‖²
start while the m×m factorisation that writes L⁻¹ still runs, each column tile once its row of
L⁻¹ is flagged final by the persistent kernel; a completion launch after the factorisation takes
the tiles the dependent launch left.  Every tile is the same product with the same K range, and
the partials are summed in the same fixed order, so every output is bitwise the one of the
sequential schedule — whatever the interleaving, the width of the factorisation (its workgroups
all resident or not: the dependent launch waits only once all of them have started, else it
leaves its tiles) or the graph path.  Reference: K20:222-234 (Q, G, big_Q) and K20:76-83
(spgp_cal_mean_and_cov), restated as the Woodbury form of DESIGN §5.
"""
import numpy as np
import pytest

import gp_oracle as O
from conftest import nrel

pytestmark = pytest.mark.gpu

KEYS_VEC = ("loo_mu", "loo_var", "pred_mu", "pred_var")
KEYS_SCAL = ("nlml", "loo_crps", "loo_logs", "logdet", "quad", "test_crps", "test_logs")


@pytest.fixture(scope="module")
def gp(gpu_ctx):
    import gpscore
    return gpscore.GP(ctx=gpu_ctx)


def _unit(gp, X, y, Xt, yt, Z, th):
    gp.set_data(X, y, kind="fitc", Z=Z)
    gp.set_test(Xt, yt)
    r = gp.fit(theta=th)
    mu, var, sc = gp.predict(with_scores=True)
    out = dict(r.objectives)
    out.update(loo_mu=r.mu_loo, loo_var=r.var_loo, pred_mu=mu, pred_var=var, **sc)
    return out


def _case(n, nt, m, d, seed):
    rng = np.random.default_rng(seed)
    X, Xt = rng.standard_normal((n, d)), rng.standard_normal((nt, d))
    Z = X[rng.choice(n, m, replace=False)]
    y, yt = np.sin(X.sum(1)), np.sin(Xt.sum(1))
    th = (0.0, np.log(1.5) * np.ones(d), np.log(0.05))
    return X, y, Xt, yt, Z, th


def _same(a, b):
    for k in KEYS_VEC:
        assert np.array_equal(a[k], b[k]), (k, nrel(a[k], b[k]))
    for k in KEYS_SCAL:
        assert float(a[k]) == float(b[k]), (k, a[k], b[k])


@pytest.mark.parametrize("n,m", [(3000, 200), (6000, 1000), (9000, 2000), (5000, 2560),
                                 (7000, 2900), (9000, 4000), (300, 250)])
def test_fitc_dep_bitwise(gp, gpu_ctx, n, m):
    """m_pad from 2 to 20 tiles (one persistent launch each: the whole q pass behind Lm's) and
    23 / 32 tiles (a recursive factorisation, C5's shape: the q pre-pass over the top L11⁻¹
    columns behind that block's launch, odd and even splits): dependent row norms on and
    off give the same bits; the oracle agrees as in the other FITC tests."""
    from gpscore import _lib
    X, y, Xt, yt, Z, th = _case(n, 700, m, 8, 31 + m)
    runs = []
    try:
        for dep in (0, 1, 1):  # (twice on: a replayed factorisation graph with signals)
            gpu_ctx.call("gps_ctx_set_option", _lib.GPS_OPT_FITC_DEP, dep)
            runs.append(_unit(gp, X, y, Xt, yt, Z, th))
    finally:
        gpu_ctx.call("gps_ctx_set_option", _lib.GPS_OPT_FITC_DEP, 1)
    _same(runs[1], runs[0])
    _same(runs[2], runs[0])
    ref = O.fast_fitc(X, y, Xt, yt, Z, *th)
    assert nrel(runs[1]["pred_mu"], ref["pred_mu"]) < 1e-6
    assert nrel(runs[1]["loo_mu"], ref["loo_mu"]) < 1e-6


@pytest.mark.parametrize("wgs", [4, 24, 256, 1024])
def test_fitc_dep_any_factorisation_width(gp, gpu_ctx, wgs):
    """Forward progress whatever the factorisation's width (GPS_OPT_DAG_WGS): 4 workgroups (a
    slow chain, the dependent launch waits long on each row), 256 or 1024 (more workgroups than
    CUs can hold beside the row-norm launch: it must leave its tiles rather than wait for
    workgroups that are not resident).  Same bits as the sequential schedule every time."""
    from gpscore import _lib
    _widths(gp, gpu_ctx, wgs, *_case(7000, 600, 2000, 8, 77))


@pytest.mark.parametrize("wgs", [4, 1024])
def test_fitc_dep_recursive_any_width(gp, gpu_ctx, wgs):
    """The same for the recursive factorisation's pre-pass (m_pad 26 tiles, L11 of 13)."""
    _widths(gp, gpu_ctx, wgs, *_case(6000, 600, 3300, 8, 78))


def _widths(gp, gpu_ctx, wgs, X, y, Xt, yt, Z, th):
    from gpscore import _lib
    try:
        gpu_ctx.call("gps_ctx_set_option", _lib.GPS_OPT_FITC_DEP, 0)
        base = _unit(gp, X, y, Xt, yt, Z, th)
        gpu_ctx.call("gps_ctx_set_option", _lib.GPS_OPT_FITC_DEP, 1)
        gpu_ctx.call("gps_ctx_set_option", _lib.GPS_OPT_DAG_WGS, wgs)
        got = _unit(gp, X, y, Xt, yt, Z, th)
    finally:
        gpu_ctx.call("gps_ctx_set_option", _lib.GPS_OPT_DAG_WGS, 0)
        gpu_ctx.call("gps_ctx_set_option", _lib.GPS_OPT_FITC_DEP, 1)
    _same(got, base)


def test_fitc_dep_eager_and_gradients(gp, gpu_ctx):
    """The dependent schedule under eager launches (GPS_OPT_GRAPH 0) and inside the gradient
    pass (gps_fitc_grad runs the same forward): values and θ / Z gradients bitwise as without."""
    from gpscore import _lib
    X, y, Xt, yt, Z, th = _case(6000, 500, 1500, 8, 5)
    outs = []
    try:
        for dep, graph in ((0, 1), (1, 0), (1, 1)):
            gpu_ctx.call("gps_ctx_set_option", _lib.GPS_OPT_FITC_DEP, dep)
            gpu_ctx.set_graphs(bool(graph))
            u = _unit(gp, X, y, Xt, yt, Z, th)
            g = gp.value_and_grad(th, objective="loo_crps")
            outs.append((u, g))
    finally:
        gpu_ctx.call("gps_ctx_set_option", _lib.GPS_OPT_FITC_DEP, 1)
        gpu_ctx.set_graphs(True)
    for u, g in outs[1:]:
        _same(u, outs[0][0])
        v0, g0, o0 = outs[0][1]
        assert g[0] == v0 and np.array_equal(g[1], g0)
        assert np.array_equal(g[2]["grad_Z"], o0["grad_Z"])
