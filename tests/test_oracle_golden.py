"""The CPU oracle (oracle/gp_oracle.py) pinned against the golden vectors that
tests/golden/make_goldens.py produced by running the reference's own helper
defs at fp64.  CPU only."""
import numpy as np
import pytest

import gp_oracle as O
import ref_torch as RT
from conftest import golden_names, load_golden, nrel, theta_of

VEC_KEYS = ("loo_mu", "loo_var", "pred_mu", "pred_var")
SCAL_KEYS = ("nlml", "loo_crps", "loo_logs", "logdet", "quad", "test_crps", "test_logs",
             "test_msll", "test_smse", "test_mse", "test_cover")

FULL = golden_names("sd_") + golden_names("full_")
FITC = golden_names("fitc_")


def _check(out, g, tol):
    for k in VEC_KEYS:
        assert nrel(out[k], g[k]) <= tol, (k, nrel(out[k], g[k]))
    for k in SCAL_KEYS:
        assert abs(out[k] - float(g[k])) <= tol * max(1.0, abs(float(g[k]))), (k, out[k], float(g[k]))


@pytest.mark.parametrize("name", FULL)
@pytest.mark.parametrize("flavour", ["ref", "fast", "torch"])
def test_full_oracle_vs_golden(name, flavour):
    """ref / fast: the numpy restatements; torch: the torch-CPU ref-mirror the bench times
    as the CPU baseline (oracle/ref_torch.py)."""
    g = load_golden(name)
    th, kind = theta_of(g)
    fn = {"ref": O.ref_full, "fast": O.fast_full, "torch": RT.ref_full}[flavour]
    out = fn(g["X"], g["y"], g["Xt"], g["yt"], *th, kind="rbf" if kind == "rbf" else "ARD")
    _check(out, g, 1e-9)


GRAD = [n for n in FULL if "grad_nlml" in load_golden(n)]


@pytest.mark.parametrize("name", GRAD)
@pytest.mark.parametrize("obj", ["nlml", "loo_crps", "loo_logs"])
def test_oracle_gradients_vs_autograd(name, obj):
    """Analytic gradients (oracle.fast_full_grad: tr(M ∂A/∂θ)) against the reference's own
    autograd `.backward()` (KF:252 / KF:339 / KF:428) captured in the goldens:
    ARD per-dimension ℓ, scalar ℓ broadcast over d, d = 1 (SIMPLE-DATA) and rbf (b = log ℓ²)."""
    g = load_golden(name)
    th, kind = theta_of(g)
    val, grad = O.fast_full_grad(g["X"], g["y"], *th, obj, kind="rbf" if kind == "rbf" else "ARD")
    assert abs(val - float(g[obj])) <= 1e-10 * max(1.0, abs(float(g[obj])))
    assert nrel(grad, g["grad_" + obj]) <= 1e-10


@pytest.mark.parametrize("name", FITC)
@pytest.mark.parametrize("flavour", ["ref", "fast", "shard3", "torch"])
def test_fitc_oracle_vs_golden(name, flavour):
    g = load_golden(name)
    th, _ = theta_of(g)
    if flavour == "ref":
        out = O.ref_fitc(g["X"], g["y"], g["Xt"], g["yt"], g["Z"], *th)
    elif flavour == "torch":
        out = RT.ref_fitc(g["X"], g["y"], g["Xt"], g["yt"], g["Z"], *th)
    else:
        out = O.fast_fitc(g["X"], g["y"], g["Xt"], g["yt"], g["Z"], *th,
                          shards=3 if flavour == "shard3" else 1)
    _check(out, g, 1e-8)


def test_l1_blocks():
    g = load_golden("l1_blocks")
    ell = g["log_ell"]
    assert nrel(O.ref_ard(g["Xa"], g["Xb"], float(g["log_sf2"]), ell), g["ard_ab"]) < 1e-14
    assert nrel(O.fast_gram(g["Xa"], g["Xb"], float(g["log_sf2"]), ell), g["ard_ab"]) < 1e-14
    assert nrel(O.fast_gram(g["Xa"], g["Xb"], float(g["iso_log_sf2"]), float(g["iso_log_ell"])),
                g["ard_iso"]) < 1e-14
    assert nrel(O.fast_gram(g["x1"], g["x2"], float(g["rbf_log_sf2"]), float(g["rbf_log_ell2"]),
                            kind="rbf"), g["rbf_12"]) < 1e-14
    assert nrel(O.ref_chol_solve(g["B"], g["A"]), g["chol_solve"]) < 1e-12
    assert nrel(O.fast_chol_solve(g["B"], g["A"]), g["chol_solve"]) < 1e-10
    assert nrel(O.ref_chol_solve(np.eye(48), g["A"]), g["chol_solve_eye"]) < 1e-12
    assert abs(O.ref_half_logdet(g["A"]) - float(g["half_logdet"])) < 1e-12
    assert nrel(O.ref_Q(g["Xa"], g["nys_Z"], g["Xb"], float(g["log_sf2"]), ell), g["Q_ab"]) < 1e-10


def test_scores():
    g = load_golden("scores")
    assert abs(O.crps(g["m"], g["c"], g["y"]) - float(g["crps"])) < 1e-14
    assert abs(O.logs(g["m"], g["c"], g["y"]) - float(g["logs"])) < 1e-14
    assert abs(O.trivial_loss(g["m"], g["c"], g["y"], g["y_train"]) - float(g["msll"])) < 1e-14
    assert abs(O.smse(g["m"], g["y"], g["y_train"]) - float(g["smse"])) < 1e-14


def test_loo_identity_bruteforce():
    """LOO closed form (KF:241-244, R&W eq. 5.12) equals refitting without point i."""
    rng = np.random.default_rng(3)
    X = rng.standard_normal((40, 3))
    y = rng.standard_normal(40)
    th = (0.2, np.log([0.9, 1.3, 2.0]), np.log(0.05))
    f = O.fast_full_fit(X, y, *th)
    for i in (0, 17, 39):
        keep = np.arange(40) != i
        A = O.fast_gram(X[keep], X[keep], th[0], th[1], diag_add=np.exp(th[2]))
        k = O.fast_gram(X[i:i + 1], X[keep], th[0], th[1]).ravel()
        mu = k @ np.linalg.solve(A, y[keep])
        var = np.exp(th[0]) + np.exp(th[2]) - k @ np.linalg.solve(A, k)
        assert abs(mu - f["loo_mu"][i]) < 1e-12
        assert abs(var - f["loo_var"][i]) < 1e-12


FITC_GRAD = [n for n in FITC if "grad_nlml" in load_golden(n)]


@pytest.mark.parametrize("name", FITC_GRAD)
@pytest.mark.parametrize("obj", ["nlml", "loo_crps", "loo_logs"])
def test_fitc_oracle_gradients_vs_autograd(name, obj):
    """Analytic O(n·m²) FITC gradients (oracle.fast_fitc_grad) against the reference's
    autograd `.backward()` through the dense n×n FITC bodies (K20:236 / K20:344 / K20:452)
    w.r.t. para_k, para_l, para_noise AND inducing_x (trained, K20:247).
    Tolerance: 1e-9 normwise when K̃mm is well conditioned; 1e-6 for the cases with
    cond(K̃mm) ≈ 5e3 (uniform Z, K20:216), where the reference's own LU solves limit agreement
    (central finite differences agree with both to ~1e-8)."""
    g = load_golden(name)
    th, _ = theta_of(g)
    val, grad, gZ = O.fast_fitc_grad(g["X"], g["y"], g["Z"], *th, obj)
    Kmm, _, _ = O.fitc_shared(g["Z"], *th[:2])
    tol = 1e-9 if np.linalg.cond(Kmm) < 1e3 else 1e-6
    assert abs(val - float(g["value_" + obj])) <= 1e-10 * max(1.0, abs(float(g["value_" + obj])))
    assert nrel(grad, g["grad_" + obj]) <= tol
    assert nrel(gZ, g["gradZ_" + obj]) <= tol


BLOCK = golden_names("block_")


@pytest.mark.parametrize("name", BLOCK)
@pytest.mark.parametrize("obj", ["dss", "kc"])
def test_blockloo_oracle_vs_golden(name, obj):
    """4-fold block-LOO DSS / KC (KF:487-543, K20:523-587, K20:655-720) composed from the
    reference's own defs: oracle value (full GP and FITC) and the full-GP analytic gradient
    against autograd."""
    g = load_golden(name)
    th, _ = theta_of(g)
    ref = float(g["value_" + obj])
    if "Z" in g:  # FITC: θ- and inducing-input gradients (K20:587 / 720, Z moved at K20:593 / 726)
        val, grad, gZ = O.fast_fitc_blockloo(g["X"], g["y"], g["Z"], *th, obj, want_grad=True)
        assert nrel(grad, g["grad_" + obj]) <= 1e-10
        assert nrel(gZ, g["gradZ_" + obj]) <= 1e-10
        assert abs(O.fast_fitc_blockloo(g["X"], g["y"], g["Z"], *th, obj) - val) <= 1e-13 * abs(val)
    else:
        val, grad = O.fast_full_blockloo(g["X"], g["y"], *th, obj, want_grad=True)
        assert nrel(grad, g["grad_" + obj]) <= 1e-10
    assert abs(val - ref) <= 1e-11 * max(1.0, abs(ref))


@pytest.mark.parametrize("name", golden_names("blockes_"))
def test_es_oracle_vs_golden(name):
    """4-fold block-LOO energy score (KF:607-663) from the reference's own ES def (KF:70-101)
    with its torch.randn draws replayed: oracle value, and the analytic gradient (the Sylvester
    solution RX + XR = Ḡ for d C^½) against autograd through torch.svd."""
    g = load_golden(name)
    th, _ = theta_of(g)
    es = {"draws": g["draws_es"], "S": int(g["num_sim"])}
    val, grad = O.fast_full_blockloo(g["X"], g["y"], *th, "es", want_grad=True, es=es)
    ref = float(g["value_es"])
    assert abs(val - ref) <= 1e-11 * max(1.0, abs(ref))
    assert nrel(grad, g["grad_es"]) <= 1e-10
    assert abs(O.fast_full_blockloo(g["X"], g["y"], *th, "es", es=es) - val) <= 1e-13 * abs(val)


def test_es_dss_single_oracle_vs_golden():
    """ES and dss of one Gaussian (KF:70-108) with the reference's draws."""
    g = load_golden("es_single")
    S, b = int(g["num_sim"]), g["C"].shape[0]
    xi = g["draws"].reshape(2, S, b)
    v = O.es_value(g["m"], g["C"], g["y"], xi[0], xi[1])
    assert abs(v - float(g["es"])) <= 1e-12 * max(1.0, abs(float(g["es"])))
    r = g["y"] - g["m"]
    d = 0.5 * b * O.LOG2PI + 0.5 * np.linalg.slogdet(g["C"])[1] + 0.5 * r @ np.linalg.solve(g["C"], r)
    assert abs(d - float(g["dss"])) <= 1e-12 * max(1.0, abs(float(g["dss"])))


@pytest.mark.parametrize("name", ["surface_cp", "surface_d2"])
def test_cp_surface_oracle_vs_golden(name):
    """contour-plot.R surfaces (CP.R:43-85): the numpy restatement against the goldens composed
    from the reference's own Python defs with CP.R's parameterisation (R parity unpinned: R is
    absent; the data are numpy draws of CP.R's generator)."""
    g = load_golden(name)
    out = O.cp_surface(g["x"], g["y"], g["ell"], g["sd"])
    for k in range(4):
        assert nrel(out[k], g["surf"][k]) < 1e-9, (k, nrel(out[k], g["surf"][k]))


@pytest.mark.parametrize("tag", ["well", "ill"])
def test_dss_k20_golden(tag):
    """K20's own dss (K20:106-111, cov_term.inverse()) and KF's (KF:103-108, chol_solve) from the
    reference's defs on the same Gaussians: the oracle's Cholesky form matches both — to 1e-13
    on the moderately conditioned covariance, and within the inverse's cond(C)·ε on the badly
    conditioned one, where the reference's two defs already differ by that much."""
    g = load_golden("dss_k20")
    m, C, y = g[f"{tag}_m"], g[f"{tag}_C"], g[f"{tag}_y"]
    b = C.shape[0]
    r = y - m
    L = np.linalg.cholesky(C)
    w = np.linalg.solve(L, r)
    d = 0.5 * b * O.LOG2PI + float(np.sum(np.log(np.diag(L)))) + 0.5 * float(w @ w)
    kf, k20 = float(g[f"{tag}_dss_kf"]), float(g[f"{tag}_dss_k20"])
    tol = 1e-13 if tag == "well" else 1e-15 * np.linalg.cond(C)
    assert abs(d - kf) <= tol * abs(kf)
    assert abs(d - k20) <= tol * abs(k20)
    assert abs(kf - k20) <= tol * abs(kf)
