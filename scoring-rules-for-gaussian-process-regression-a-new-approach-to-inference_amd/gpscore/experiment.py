"""Data ingest and the replicate harness of the reference scripts, on top of the device hot
path.

kin40k-FULL-compare.py (KF) loops over TT replicates (KF:149-190): 800 of the 10 000
training rows drawn with Python's `random` seeded 100·j (KF:194-196), 300 of them held out
for validation (KF:203-209), the first 500 test rows (KF:199-200); then five fits of the
full GP from a random start, each scored on the test set (MSE, SMSE, LogS, CRPS, MSLL and
the ±2σ coverage, e.g. KF:267-299).  KIN40K-COMPARE-ALL-FITC-20.py (K20) does the same with
a 20-point FITC model whose inducing inputs are trained too, drawing rows without
reseeding (K20:184-192).

Every number here comes from gpscore.GP (libgpscore.so): the SGD loops are GP.train, the
predictive and its scores GP.predict.  The workbook is not shipped (the scripts open it from
a Windows drive), so load_sheets reads the .xlsx when pandas has an Excel engine, or the
same four sheets from an .npz or a directory of <sheet>.csv files.
"""
from __future__ import annotations

import os
import random
from dataclasses import dataclass

import numpy as np

from ._lib import NotPositiveDefinite
from .gp import GP

SHEETS = ("trainx", "trainy", "testx", "testy")
METRICS = ("mse", "smse", "logs", "crps", "msll", "cover")


def _as2d(a):
    a = np.asarray(a, dtype=np.float64)
    return a.reshape(a.shape[0], -1) if a.ndim == 1 else a


def load_sheets(path):
    """{trainx, trainy, testx, testy} as 2-D float64 arrays from kin40k.xlsx (sheet names and
    header=None as KF:197-200), an .npz holding those keys, or a directory of <sheet>.csv."""
    if os.path.isdir(path):
        return {s: _as2d(np.loadtxt(os.path.join(path, s + ".csv"), delimiter=",", ndmin=2))
                for s in SHEETS}
    if str(path).endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return {s: _as2d(z[s]) for s in SHEETS}
    import pandas as pd  # an Excel engine (openpyxl / xlrd) must be installed for .xlsx
    return {s: _as2d(pd.read_excel(path, sheet_name=s, header=None).values) for s in SHEETS}


def synthetic_sheets(rng=None, n_pool=10000, n_test=500, d=8):
    """Stand-in sheets of kin40k's shapes (d = 8 inputs, one target) from the SURVEY.md §8d
    generator, for running the harness without the workbook."""
    rng = np.random.default_rng(rng)
    w = rng.standard_normal(d) / np.sqrt(d)
    X, Xt = rng.standard_normal((n_pool, d)), rng.standard_normal((n_test, d))
    y = np.sin(3 * X @ w) + 0.1 * rng.standard_normal(n_pool)
    yt = np.sin(3 * Xt @ w) + 0.1 * rng.standard_normal(n_test)
    return {"trainx": X, "trainy": y[:, None], "testx": Xt, "testy": yt[:, None]}


def replicate_indices(j=None, n_pool=10000, n_train=500, num_va=300, rs=None):
    """Row draws of replicate j as the scripts make them with the global `random`:
    random.seed(100·j) (KF:194; K20 never reseeds: pass j=None and one `rs` for all
    replicates), sam = random.sample(range(0, n_pool), n_train + num_va) (KF:196),
    va = random.sample(range(0, n_train + num_va), num_va) (KF:203)."""
    if rs is None:
        rs = random.Random()
    if j is not None:
        rs.seed(j * 100)
    sam = np.array(rs.sample(range(0, n_pool), n_train + num_va))
    va = np.array(rs.sample(range(0, n_train + num_va), num_va))
    return sam, va


def replicate(sheets, j=None, n_train=500, num_va=300, n_test=500, n_pool=10000, rs=None):
    """Train / validation / test arrays of replicate j (KF:194-211): full = trainx[sam], the va
    rows held out (np.delete, KF:208-209), test = the first n_test rows (KF:199-200)."""
    sam, va = replicate_indices(j, n_pool, n_train, num_va, rs)
    full_x, full_y = sheets["trainx"][sam], sheets["trainy"][sam]
    return {"train_x": np.delete(full_x, va, axis=0),
            "train_y": np.delete(full_y, va, axis=0).ravel(),
            "va_x": full_x[va], "va_y": full_y[va].ravel(),
            "test_x": sheets["testx"][:n_test], "test_y": sheets["testy"][:n_test].ravel()}


@dataclass(frozen=True)
class Method:
    """One fit of the scripts: objective (GP.train name), SGD length and step, starting point,
    the lines it restates."""
    objective: str
    itr: int
    lr: float
    lr_z: float | None = None  # FITC inducing-input step (None: lr)
    init: str = "rand_l"       # rand3: para_l ~ U(0,1)^d, para_k, para_noise ~ U(0,1) (KF:226-233)
                               # rand_l: para_l ~ U(0,1)^d, para_k = para_noise = 1 (KF:321-324)
                               # ones: scalar para_l = para_k = para_noise = 1 (K20:422-424)
    z_init: str = "rand"       # FITC inducing_x start: U(0,1) (K20:215) or N(0,1) (K20:531)
    ref: str = ""


KF_METHODS = {
    "crps": Method("loo_crps", 400, 1.0, init="rand3", ref="KF:220-299"),
    "nlml": Method("nlml", 400, 5e-4, ref="KF:312-399"),   # the scripts' "gp" series
    "logs": Method("loo_logs", 500, 0.05, ref="KF:405-482"),
    "dss": Method("dss", 150, 1e-3, ref="KF:487-601"),
    "es": Method("es", 25, 0.1, ref="KF:607-732"),
}
K20_METHODS = {
    "crps": Method("loo_crps", 2000, 1.0, 1.0, ref="K20:207-247"),
    "nlml": Method("nlml", 3000, 1e-4, 1e-3, ref="K20:315-350"),
    "logs": Method("loo_logs", 3000, 0.2, 0.2, init="ones", ref="K20:417-458"),
    "dss": Method("dss", 3000, 1e-3, 1e-3, z_init="randn", ref="K20:523-593"),
    "kc": Method("kc", 3000, 0.1, 0.1, ref="K20:655-726"),
}


def initial_theta(method, d, rng):
    """(para_k, para_l, para_noise) at the method's start (torch.rand there, numpy here)."""
    if method.init == "rand3":
        return (float(rng.random()), rng.random(d), float(rng.random()))
    if method.init == "ones":
        return (1.0, np.array([1.0]), 1.0)
    return (1.0, rng.random(d), 1.0)


def run_method(gp, data, method, rng, kind="full", m=20, itr=None, stale_noise=True,
               num_sim=300):
    """One fit (the method's SGD loop, GP.train) + test predictive + score bundle.
    Returns {mse, smse, logs, crps, msll, cover, theta, Z, failed}.  The predictive uses the
    final kernel parameters and, with stale_noise, the noise variance of the last iteration's
    forward pass: the scripts' module-global sigma_noise_sq is set before the last update and
    read by cal_mean_and_cov / spgp_cal_mean_and_cov.  The ES and KC fits turn
    a non-PD factorisation into zero metrics (KF:726-732, K20:784-790); others raise."""
    d = data["train_x"].shape[1]
    th0 = initial_theta(method, d, rng)
    itr = method.itr if itr is None else int(itr)
    block_kw = {"num_sim": num_sim, "rng": rng} if method.objective == "es" else None
    Z0 = None
    if kind == "fitc":
        Z0 = rng.random((m, d)) if method.z_init == "rand" else rng.standard_normal((m, d))
    try:
        theta, series = gp.train(th0, method.objective, lr=method.lr, itr=itr,
                                 X=data["train_x"], y=data["train_y"], Z0=Z0, lr_z=method.lr_z,
                                 block_kw=block_kw)
        noise = theta[2]
        if stale_noise:
            noise = float(series["theta"][itr - 2][-1]) if itr >= 2 else float(th0[2])
        gp.fit(theta=(theta[0], theta[1], noise), return_loo=False)
        _, _, sc = gp.predict(data["test_x"], data["test_y"], with_scores=True)
    except NotPositiveDefinite:
        if method.objective not in ("es", "kc"):
            raise
        return dict({k: 0.0 for k in METRICS}, theta=None, Z=None, failed=True)
    return {"mse": sc["test_mse"], "smse": sc["test_smse"], "logs": sc["test_logs"],
            "crps": sc["test_crps"], "msll": sc["test_msll"], "cover": sc["test_cover"],
            "theta": theta, "Z": series.get("Z"), "failed": False}


def run(sheets, TT=30, methods=None, kind="full", itr=None, seed=None, ctx=None, reseed=True,
        **kw):
    """TT replicates → {method: {metric: array(TT)}}, the scripts' <metric>_<method>_series
    (KF:149-184, K20:145-180).  reseed: KF's random.seed(100·j); False: one unseeded stream
    (K20).  `seed` drives the random starting points (torch.rand in the scripts)."""
    methods = methods or (KF_METHODS if kind == "full" else K20_METHODS)
    gp = GP(ctx=ctx)
    rng = np.random.default_rng(seed)
    rs = None if reseed else random.Random()
    out = {name: {k: np.zeros(TT) for k in METRICS} for name in methods}
    n_pool = sheets["trainx"].shape[0]  # 10 000 in kin40k, the scripts' range(0, 10000)
    for j in range(TT):
        data = replicate(sheets, j if reseed else None, n_pool=n_pool, rs=rs)
        for name, meth in methods.items():
            r = run_method(gp, data, meth, rng, kind=kind, itr=itr, **kw)
            for k in METRICS:
                out[name][k][j] = r[k]
    return out
