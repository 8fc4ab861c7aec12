"""High-level facade: fit / predict / score on numpy arrays.

    gp = gpscore.GP()                             # one device context
    res = gp.fit(X, y, theta)                     # full GP  (KF:239-245, 329-334, 416-424)
    res = gp.fit(X, y, theta, kind="fitc", Z=Z)   # FITC     (K20:222-234, 329-340, 434-447)
    mu, var = gp.predict(Xt)                      # cal_mean_and_cov / spgp_cal_mean_and_cov, diag
    sc = gp.score(mu, var, yt, y)                 # crps, logs, trivial_loss, SMSE, MSE, coverage

``theta = (log_sf2, log_ell, log_sn2)`` uses the reference's log-parameterisation
(para_k, para_l, para_noise): ``log_ell`` is a scalar or a length-d vector
(ARD, b = log ℓ, KF:8-12); with ``rbf=True`` it is log ℓ² (SD:8-21).

Every number is computed by libgpscore.so on the GPU; there is no CPU path.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import (GPS_ARD, GPS_RBF, GPS_SURF_LOGS_ADD_NOISE, OBJ_NAMES, SCORE_NAMES,
                   SURFACE_NAMES, f64, ptr)

BLOCK_OBJS = ["dss", "kc", "es"]  # GPS_BLOCK_DSS, GPS_BLOCK_KC, GPS_BLOCK_ES


def es_draws(n, nfold=4, num_sim=300, rng=None):
    """Standard-normal draws of the block-LOO energy score in the C-ABI's layout: fold f (rows
    [int(f·n/k), int((f+1)·n/k)), KF:496-499) holds ξ_f then ξ'_f, each num_sim × b_f — the
    two torch.randn(num_sim, shape1) calls of ES (KF:79-80) in the scripts' fold order.
    ``rng``: a numpy Generator, a seed, or None (fresh entropy, as the scripts re-draw)."""
    rng = np.random.default_rng(rng)
    bnd = [0] + [int(f * n / nfold) for f in range(1, nfold)] + [n]
    return np.concatenate([rng.standard_normal(2 * num_sim * (b - a))
                           for a, b in zip(bnd[:-1], bnd[1:])])


def pack_theta(theta, d):
    """[log_sf2, log_ell..., log_sn2] as the C-ABI expects; returns (array, n_ell)."""
    log_sf2, log_ell, log_sn2 = theta
    ell = np.atleast_1d(np.asarray(log_ell, dtype=np.float64)).ravel()
    if ell.size not in (1, d):
        raise ValueError(f"log_ell has {ell.size} entries, expected 1 or d={d}")
    t = np.concatenate([[float(np.asarray(log_sf2).ravel()[0])], ell,
                        [float(np.asarray(log_sn2).ravel()[0])]])
    return np.ascontiguousarray(t), int(ell.size)


@dataclass
class FitResult:
    kind: str
    objectives: dict
    mu_loo: np.ndarray | None = None
    var_loo: np.ndarray | None = None
    extra: dict = field(default_factory=dict)

    def __getitem__(self, k):
        return self.objectives[k]


class GP:
    """Device-resident GP hot path (one context = one GPU + one HIP stream)."""

    def __init__(self, ctx: _lib.Context | None = None, device: int | None = None):
        if ctx is None:
            ctx = _lib.Context(device) if device is not None else _lib.default_context()
        self.ctx = ctx
        self.kind = None
        self._X = self._Z = None
        self._Xt = self._yt = None
        self._train_key = self._test_key = self._z_key = None
        self._token = object()  # identifies this GP's data in ctx.resident
        self.comm = None  # set by gpscore.dist.attach_comm
        self.n_total = None
        self.nt_total = None
        self.ytr_stats = None  # (mean, unbiased var) over ALL ranks' training targets

    # ------------------------------------------------------------------ data
    def set_data(self, X, y, kind="full", Z=None, n_total=None, ytr_stats=None):
        X, y = f64(X, 2), f64(y).ravel()
        if X.shape[0] != y.size:
            raise ValueError("X and y disagree on n")
        n, d = X.shape
        self.kind = kind
        self._X, self._y = X, y
        if kind == "full":
            self.ctx.call("gps_full_set_data", ptr(X), ptr(y), n, d)
            self.ctx.resident[kind] = self._token
            self._Xt = self._yt = None
        elif kind == "fitc":
            self.n_total = n if n_total is None else int(n_total)
            if ytr_stats is None:
                ytr_stats = (float(y.mean()), float(y.var(ddof=1)) if n > 1 else 1.0)
            self.ytr_stats = ytr_stats
            self.ctx.call("gps_fitc_set_data", ptr(X), ptr(y), n, d, ytr_stats[0], ytr_stats[1],
                          self.n_total)
            self.ctx.resident[kind] = self._token
            self._Xt = self._yt = None
            if Z is not None:
                self.set_inducing(Z)
        else:
            raise ValueError("kind must be 'full' or 'fitc'")
        self._train_key = (id(X), X.shape)
        return self

    def set_inducing(self, Z):
        Z = f64(Z, 2)
        if self._X is not None and Z.shape[1] != self._X.shape[1]:
            raise ValueError("Z and X disagree on d")
        self._Z = Z
        self._ensure_resident()
        self.ctx.call("gps_fitc_set_inducing", ptr(Z), Z.shape[0])

    def set_test(self, Xt, yt=None, nt_total=None):
        Xt = f64(Xt, 2)
        yt = None if yt is None else f64(yt).ravel()
        nt = Xt.shape[0]
        self._ensure_resident()
        if self.kind == "full":
            self.ctx.call("gps_full_set_test", ptr(Xt), ptr(yt), nt)
        else:
            self.nt_total = nt if nt_total is None else int(nt_total)
            self.ctx.call("gps_fitc_set_test", ptr(Xt), ptr(yt), nt, self.nt_total)
        self._nt = nt
        self._has_yt = yt is not None
        self._Xt, self._yt = Xt, yt

    def _ensure_resident(self):
        """Several GP objects may share one context, whose device holds ONE full-GP and ONE
        FITC data set: if another GP uploaded since, put this one's data (and inducing and
        test points) back.  The factor of a fit is not restored — predict then needs a new
        fit, as after any set_data."""
        if self.kind is None or self.ctx.resident.get(self.kind) is self._token:
            return
        X, y, n, d = self._X, self._y, self._X.shape[0], self._X.shape[1]
        if self.kind == "full":
            self.ctx.call("gps_full_set_data", ptr(X), ptr(y), n, d)
            if self._Xt is not None:
                self.ctx.call("gps_full_set_test", ptr(self._Xt), ptr(self._yt), self._Xt.shape[0])
        else:
            self.ctx.call("gps_fitc_set_data", ptr(X), ptr(y), n, d, self.ytr_stats[0],
                          self.ytr_stats[1], self.n_total)
            if self._Z is not None:
                self.ctx.call("gps_fitc_set_inducing", ptr(self._Z), self._Z.shape[0])
            if self._Xt is not None:
                self.ctx.call("gps_fitc_set_test", ptr(self._Xt), ptr(self._yt), self._Xt.shape[0],
                              self.nt_total)
        self.ctx.resident[self.kind] = self._token

    # ------------------------------------------------------------------- fit
    def fit(self, X=None, y=None, theta=(0.0, 0.0, 0.0), kind="full", Z=None, rbf=False,
            return_loo=True):
        """One forward evaluation of the reference's per-iteration objective bodies
        at theta.  Returns objectives {nlml, loo_crps, loo_logs, logdet, quad} and
        the LOO predictive mean / variance (R&W eq. 5.12)."""
        if X is not None:
            self.set_data(X, y, kind=kind, Z=Z)
        elif Z is not None:
            self.set_inducing(Z)
        if self.kind is None:
            raise ValueError("no training data")
        self._ensure_resident()
        d = self._X.shape[1]
        th, n_ell = pack_theta(theta, d)
        obj = np.zeros(5)
        n = self._X.shape[0]
        mu = np.empty(n) if return_loo else None
        var = np.empty(n) if return_loo else None
        if self.kind == "full":
            self.ctx.call("gps_full_fit", GPS_RBF if rbf else GPS_ARD, ptr(th), n_ell, ptr(obj),
                          ptr(mu), ptr(var))
        else:
            if rbf:
                raise ValueError("FITC uses the ARD kernel (K20:32-39)")
            if self._Z is None:
                raise ValueError("FITC needs inducing points Z")
            self.ctx.call("gps_fitc_fit", ptr(th), n_ell, ptr(obj), ptr(mu), ptr(var))
        return FitResult(self.kind, dict(zip(OBJ_NAMES, obj.tolist())), mu, var)

    # ------------------------------------------------------------- gradients
    def value_and_grad(self, theta, objective="loo_crps", X=None, y=None, rbf=False, Z=None,
                       **block_kw):
        """Objective value and its analytic gradient at theta — the forward body plus the
        `.backward()` of one GD iteration of the reference (full GP: KF:239-252 LOO-CRPS,
        KF:329-339 NLML, KF:416-428 LOO-LogS, KF:487-543 DSS, KF:607-663 ES; FITC:
        K20:222-236, 329-344, 434-452, 523-587 DSS, 655-720 KC).
        Returns (value, grad, objectives) with grad = [d/d para_k, d/d para_l (1 or d),
        d/d para_noise]; for FITC ``objectives["grad_Z"]`` holds d/d inducing_x (m×d),
        the inducing inputs being trained parameters there (K20:247).  ``block_kw`` goes to
        block_loo (nfold, num_sim, beta, draws, rng)."""
        if X is not None:
            self.set_data(X, y, kind="fitc" if Z is not None else "full", Z=Z)
        elif Z is not None:
            self.set_inducing(Z)
        if objective in BLOCK_OBJS:
            res = self.block_loo(theta, objective, grad=True, rbf=rbf, **block_kw)
            objs = {objective: res[0], "folds": res[2]}
            if self.kind == "fitc":
                objs["grad_Z"] = res[3]
            return res[0], res[1], objs
        if objective not in OBJ_NAMES[:3]:
            raise ValueError(f"objective must be one of {OBJ_NAMES[:3] + BLOCK_OBJS}")
        self._ensure_resident()
        th, n_ell = pack_theta(theta, self._X.shape[1])
        obj = np.zeros(5)
        grad = np.zeros(2 + n_ell)
        if self.kind == "fitc":
            if rbf:
                raise ValueError("FITC uses the ARD kernel (K20:32-39)")
            if self._Z is None:
                raise ValueError("FITC needs inducing points Z")
            gz = np.zeros_like(self._Z)
            self.ctx.call("gps_fitc_grad", ptr(th), n_ell, OBJ_NAMES.index(objective), ptr(obj),
                          ptr(grad), ptr(gz))
            objs = dict(zip(OBJ_NAMES, obj.tolist()))
            objs["grad_Z"] = gz
            return objs[objective], grad, objs
        self.ctx.call("gps_full_grad", GPS_RBF if rbf else GPS_ARD, ptr(th), n_ell,
                      OBJ_NAMES.index(objective), ptr(obj), ptr(grad))
        objs = dict(zip(OBJ_NAMES, obj.tolist()))
        return objs[objective], grad, objs

    def block_loo(self, theta, objective="dss", nfold=4, grad=False, rbf=False, num_sim=300,
                  beta=1.0, draws=None, rng=None):
        """k-fold block leave-out objective at theta, summed over the
        folds as the scripts do: "dss" — the Dawid-Sebastiani score of each fold's block-LOO
        predictive (full GP KF:487-543, FITC K20:523-587); "kc" — the fold-mean CRPS of its
        marginals (K20:655-720); "es" — the energy score of the fold's multivariate predictive
        (full GP, ES KF:70-101 in the loop KF:607-663) from num_sim draws per fold: pass
        ``draws`` (es_draws layout) to fix them, else they are drawn from ``rng`` (the scripts
        re-draw torch.randn on every call).
        Returns value, or with grad=True (value, grad, per-fold values) — the `.backward()` at
        KF:543 / 663 — and for FITC also d/d inducing_x: (value, grad, folds, grad_Z)."""
        if objective not in BLOCK_OBJS:
            raise ValueError(f"objective must be one of {BLOCK_OBJS}")
        self._ensure_resident()
        n, d = self._X.shape
        th, n_ell = pack_theta(theta, d)
        val = np.zeros(1)
        folds = np.zeros(nfold)
        code = BLOCK_OBJS.index(objective)
        g = np.zeros(2 + n_ell) if grad else None
        if self.kind == "fitc":
            if objective == "es":
                raise ValueError("the energy score is a full-GP objective (KF:607-663)")
            gz = np.zeros_like(self._Z) if grad else None
            self.ctx.call("gps_fitc_blockloo", ptr(th), n_ell, nfold, code, ptr(val), ptr(g),
                          ptr(gz), ptr(folds))
            return (float(val[0]), g, folds, gz) if grad else float(val[0])
        kind = GPS_RBF if rbf else GPS_ARD
        if objective == "es":
            if draws is None:
                draws = es_draws(n, nfold, num_sim, rng)
            draws = f64(draws).ravel()
            if draws.size != 2 * num_sim * n:
                raise ValueError(f"draws must hold 2·num_sim·n = {2 * num_sim * n} values")
            self.ctx.call("gps_full_blockloo_es", kind, ptr(th), n_ell, nfold, int(num_sim),
                          float(beta), ptr(draws), ptr(val), ptr(g), ptr(folds))
        else:
            self.ctx.call("gps_full_blockloo", kind, ptr(th), n_ell, nfold, code, ptr(val), ptr(g),
                          ptr(folds))
        return (float(val[0]), g, folds) if grad else float(val[0])

    def train(self, theta0, objective="loo_crps", lr=1.0, itr=400, X=None, y=None, rbf=False,
              callback=None, Z0=None, lr_z=None, block_kw=None):
        """The reference's GD fit loop: `itr` plain SGD steps para -= lr * grad on
        (para_k, para_l, para_noise) — full GP e.g. KF:236-260 — one forward + analytic
        backward per step on the device.  FITC (K20:219-251, 324-354, 428-458) also moves
        the inducing inputs: inducing_x -= lr_z * grad_Z (lr_z defaults to lr; the
        reference uses 1 / 0.001 / 0.2 for LOO-CRPS / NLML / LOO-LogS, K20:221, 327, 431).
        Returns (theta, series); series holds the objective value before each step, the
        parameters after it and, for FITC, the final inducing inputs under "Z"."""
        if X is not None:
            self.set_data(X, y, kind="fitc" if Z0 is not None else "full", Z=Z0)
        elif Z0 is not None:
            self.set_inducing(Z0)
        d = self._X.shape[1]
        th, n_ell = pack_theta(theta0, d)
        th = th.copy()
        fitc = self.kind == "fitc"
        lr_z = lr if lr_z is None else lr_z
        Z = self._Z.copy() if fitc else None
        values = np.zeros(itr)
        params = np.zeros((itr, th.size))
        for i in range(itr):
            val, g, objs = self.value_and_grad((th[0], th[1:1 + n_ell], th[-1]), objective,
                                               rbf=rbf, **(block_kw or {}))
            values[i] = val
            th -= lr * g
            params[i] = th
            if fitc:
                Z -= lr_z * objs["grad_Z"]
                self.set_inducing(Z)
            if callback is not None:
                callback(i, val, th)
        theta = (float(th[0]), th[1:1 + n_ell].copy(), float(th[-1]))
        series = {"objective": values, "theta": params}
        if fitc:
            series["Z"] = Z
        return theta, series

    # --------------------------------------------------------------- predict
    def predict(self, Xt=None, yt=None, with_scores=False):
        """Predictive mean and variance (the diagonal of cal_mean_and_cov /
        spgp_cal_mean_and_cov) at Xt with the last fit's factorisation."""
        if Xt is not None:
            self.set_test(Xt, yt)
        self._ensure_resident()
        nt = self._nt
        mu, var, sc = np.empty(nt), np.empty(nt), np.zeros(6)
        name = "gps_full_predict" if self.kind == "full" else "gps_fitc_predict"
        self.ctx.call(name, ptr(mu), ptr(var), ptr(sc))
        if with_scores:
            return mu, var, dict(zip(SCORE_NAMES, sc.tolist()))
        return mu, var

    # ----------------------------------------------------------------- score
    def score(self, mu, var, y_test, y_train):
        """crps, logs, trivial_loss (MSLL), SMSE, MSE and ±2σ coverage (KF:276-292)."""
        return score(mu, var, y_test, y_train, ctx=self.ctx)


def score(mu, var, y_test, y_train, ctx=None):
    ctx = ctx or _lib.default_context()
    mu, var, yt = f64(mu).ravel(), f64(var).ravel(), f64(y_test).ravel()
    ytr = f64(y_train).ravel()
    out = np.zeros(6)
    ctx.call("gps_scores", ptr(mu), ptr(var), ptr(yt), yt.size, float(ytr.mean()),
             float(ytr.var(ddof=1)), ptr(out))
    return dict(zip(SCORE_NAMES, out.tolist()))


def fit(X, y, theta, kind="full", Z=None, rbf=False, ctx=None):
    return GP(ctx).fit(X, y, theta, kind=kind, Z=Z, rbf=rbf)


def surface(X, y, ell_grid, noise_sd_grid, log_sf2=0.0, logs_add_noise=True, ctx=None):
    """The objective surfaces of contour-plot.R (CP.R:43-85) over a length-scale × noise grid,
    one small full GP per grid point on the device (n <= 128: one wavefront each; beyond that
    one resident fit per point, and X, y become the context's full-GP data).

    ``ell_grid`` holds length-scales ℓ (not logs; CP.R's ``l``), ``noise_sd_grid`` noise
    standard deviations s entering as s² (CP.R's ``j``); the kernel is
    exp(log_sf2)·exp(−½‖x − x'‖²/ℓ²) (CP.R:15-23 with k² = exp(log_sf2)).  Returns a dict of
    (len(noise_sd_grid), len(ell_grid)) arrays — rows noise, columns length-scale, as R's
    ``matrix(…, nrow = 50)`` (CP.R:113-141): "loo_crps" (cal_m_crps CP.R:43-53),
    "insample_crps" (wrong_cal_m_crps CP.R:55-64), "nlml" (cal_NLML CP.R:68-73), "loo_logs"
    (cal_m_logs CP.R:75-85; its LOO variance carries + s² as CP.R:81 writes it unless
    ``logs_add_noise`` is False)."""
    ctx = ctx or _lib.default_context()
    X = f64(X, 2)
    y = f64(y).ravel()
    if X.shape[0] != y.size:
        raise ValueError("X and y disagree on n")
    ell = f64(ell_grid).ravel()
    sd = f64(noise_sd_grid).ravel()
    out = np.empty((4, sd.size, ell.size))
    ctx.call("gps_full_surface", ptr(X), ptr(y), y.size, X.shape[1], float(log_sf2), ptr(ell),
             ell.size, ptr(sd), sd.size, GPS_SURF_LOGS_ADD_NOISE if logs_add_noise else 0, ptr(out))
    return dict(zip(SURFACE_NAMES, out))
