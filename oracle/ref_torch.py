"""CPU ORACLE (torch flavour) — test infrastructure only, never the product path.

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg may import this module, as the
checker and as the timed CPU baseline.  It restates the reference's op sequence in the
reference's own framework — PyTorch CPU tensors in float64 — the way SURVEY.md §8(d) /
BASELINE.md ("ref-mirror, torch-CPU fp64") plans the baseline: every ``chol_solve`` is an
UPPER Cholesky followed by two general LU solves (KF:25-29: torch 0.4's ``potrf`` →
``torch.linalg.cholesky(upper=True)``, ``gesv`` → ``torch.linalg.solve``, LAPACK
getrf + getrs), recomputed on every call as the scripts do; the ARD Gram by the
``2·x·x'ᵀ − ‖x‖² − ‖x'‖²`` expansion (KF:7-23); the LOO diagonal via
``chol_solve(I, A)`` (KF:242); the predictive covariance materialised in full
(cal_mean_and_cov KF:121-126, spgp_cal_mean_and_cov K20:76-83); FITC dense n×n
(K20:222-234, 329-340, 434-447).

Pinned: ``tests/test_oracle_golden.py`` checks it against the golden vectors that
``tests/golden/make_goldens.py`` produced from the reference's own helper defs.
Aliases: KF = kin40k-FULL-compare.py, K20 = KIN40K-COMPARE-ALL-FITC-20.py,
SD = "SIMPLE-DATA FULL-comapre.py".
"""
from __future__ import annotations

import math

import numpy as np
import torch

LOG2PI = math.log(2.0 * math.pi)
JITTER = 1e-3  # KF:36


def _t(a):
    return torch.as_tensor(np.asarray(a, np.float64))


def ard(x, xp, log_sf2, log_ell, kind="ARD"):
    """KF:7-23 (ARD, b = log ℓ) / SD:8-21 (rbf, b = log ℓ²): scale the inputs by the
    length-scales, res = 2·x·x'ᵀ − ‖x‖² − ‖x'‖², K = sf²·exp(½ res)."""
    d = x.shape[1]
    b = _t(np.atleast_1d(log_ell)).view(1, -1)
    ell = torch.exp(b) if kind == "ARD" else torch.exp(0.5 * b)
    if ell.numel() == 1:
        ell = ell.expand(1, d)
    xs, xps = x / ell, xp / ell
    res = 2.0 * xs @ xps.T
    res = res - (xs * xs).sum(1, keepdim=True) - (xps * xps).sum(1).view(1, -1)
    return math.exp(float(log_sf2)) * torch.exp(0.5 * res)


def chol_solve(B, A):
    """KF:25-29: c = potrf(A) (upper); s1 = gesv(B, cᵀ); s2 = gesv(s1, c)."""
    c = torch.linalg.cholesky(A, upper=True)
    s1 = torch.linalg.solve(c.T, B)
    return torch.linalg.solve(c, s1)


def half_logdet(A):
    """KF:332: potrf(A).diag().log().sum()."""
    return torch.linalg.cholesky(A, upper=True).diagonal().log().sum()


def crps(m, c, y):
    """KF:60-68 (c is the VARIANCE)."""
    s = c.sqrt()
    z = (y - m) / s
    cdf = 0.5 * (1.0 + torch.erf(z / math.sqrt(2.0)))
    pdf = (1.0 / math.sqrt(2.0 * math.pi)) * torch.exp(-z * z / 2.0)
    return (s * (z * (2.0 * cdf - 1.0) + 2.0 * pdf - 1.0 / math.sqrt(math.pi))).mean()


def logs(m, c, y):
    """KF:52-57."""
    return ((y - m) ** 2 / (2.0 * c) + c.sqrt().log() + 0.5 * LOG2PI).mean()


def scores(mu, var, yt, y):
    """KF:276-292: MSE, SMSE (KF:128-134), LogS, CRPS, MSLL (trivial_loss KF:110-119,
    unbiased train variance) and ±2σ coverage."""
    sd = var.sqrt()
    mean_y, var_y = y.mean(), y.var()  # torch's var() is the unbiased one (KF:114)
    logs_sum = (yt - mu) ** 2 / (2.0 * var) + sd.log() + 0.5 * LOG2PI
    triv = 0.5 * torch.log(2.0 * math.pi * var_y) + (yt - mean_y) ** 2 / (2.0 * var_y)
    cover = (((mu + 2 * sd - yt) > 0) & ((yt - (mu - 2 * sd)) > 0)).double().mean()
    return {"test_mse": float(((mu - yt) ** 2).mean()),
            "test_smse": float(((mu - yt) ** 2).mean() / ((mean_y - yt) ** 2).mean()),
            "test_logs": float(logs(mu, var, yt)), "test_crps": float(crps(mu, var, yt)),
            "test_msll": float((logs_sum - triv).mean()), "test_cover": float(cover)}


def ref_full(X, y, Xt, yt, log_sf2, log_ell, log_sn2, kind="ARD"):
    """The full-GP unit the bench times, in the scripts' op order: LOO-CRPS body KF:239-245,
    NLML body KF:329-334, LOO-LogS body KF:416-424 (same LOO vectors), predict + score
    KF:365-391 with the full n*×n* covariance (cal_mean_and_cov, KF:121-126)."""
    X, Xt = _t(X), _t(Xt)
    y, yt = _t(y).view(-1, 1), _t(yt).view(-1, 1)
    n = y.shape[0]
    sn2 = math.exp(float(log_sn2))
    k_ff = ard(X, X, log_sf2, log_ell, kind)
    big_k = k_ff + sn2 * torch.eye(n, dtype=torch.float64)
    kii = torch.diag(chol_solve(torch.eye(n, dtype=torch.float64), big_k)).view(n, 1)
    mu_loo = y - chol_solve(y, big_k) / kii
    var_loo = 1.0 / kii
    hl = half_logdet(big_k)
    quad = float(y.T @ chol_solve(y, big_k))
    k_sf = ard(Xt, X, log_sf2, log_ell, kind)
    k_ss = ard(Xt, Xt, log_sf2, log_ell, kind)
    nt = k_sf.shape[0]
    mu = k_sf @ chol_solve(y, big_k)
    cov = sn2 * torch.eye(nt, dtype=torch.float64) + k_ss - k_sf @ chol_solve(k_sf.T, big_k)
    var = torch.diag(cov).view(-1, 1)
    out = {"loo_mu": mu_loo.ravel().numpy(), "loo_var": var_loo.ravel().numpy(),
           "loo_crps": float(crps(mu_loo, var_loo, y)), "loo_logs": float(logs(mu_loo, var_loo, y)),
           "nlml": 0.5 * n * LOG2PI + float(hl) + 0.5 * quad, "logdet": 2.0 * float(hl),
           "quad": quad, "pred_mu": mu.ravel().numpy(), "pred_var": var.ravel().numpy()}
    out.update(scores(mu, var, yt, y))
    return out


def ref_Q(a, u, b, log_sf2, log_ell):
    """KF:32-39: K_au · chol_solve(K_ub, K_uu + 1e-3·I)."""
    K_uu = ard(u, u, log_sf2, log_ell) + JITTER * torch.eye(u.shape[0], dtype=torch.float64)
    return ard(a, u, log_sf2, log_ell) @ chol_solve(ard(u, b, log_sf2, log_ell), K_uu)


def ref_fitc(X, y, Xt, yt, Z, log_sf2, log_ell, log_sn2):
    """Dense reference FITC, one unit: LOO-CRPS body K20:222-234, LOO-LogS variance
    K20:442-447, NLML K20:329-340 and predict + score K20:270-296 (spgp_cal_mean_and_cov
    K20:76-83).  O(n³) time and an n×n matrix, as the scripts."""
    X, Xt, Z = _t(X), _t(Xt), _t(Z)
    y, yt = _t(y).view(-1, 1), _t(yt).view(-1, 1)
    n = y.shape[0]
    sn2 = math.exp(float(log_sn2))
    eye = torch.eye(n, dtype=torch.float64)
    k_ff = ard(X, X, log_sf2, log_ell)
    Q_ff = ref_Q(X, Z, X, log_sf2, log_ell)
    G = torch.diag(k_ff - Q_ff + sn2 * eye) * eye
    big_Q = Q_ff + G
    qii = torch.diag(chol_solve(eye, big_Q)).view(n, 1)
    mu_loo = y - chol_solve(y, big_Q) / qii
    var_loo = 1.0 / qii
    var_logs = 1.0 / qii + sn2 - torch.diag(big_Q).view(n, 1) + torch.diag(k_ff).view(n, 1)
    hl = half_logdet(big_Q)
    quad = float(y.T @ chol_solve(y, big_Q))
    Q_sf = ref_Q(Xt, Z, X, log_sf2, log_ell)
    k_ss = ard(Xt, Xt, log_sf2, log_ell)
    nt = Q_sf.shape[0]
    mu = Q_sf @ chol_solve(y, big_Q)
    cov = sn2 * torch.eye(nt, dtype=torch.float64) + k_ss - Q_sf @ chol_solve(Q_sf.T, big_Q)
    var = torch.diag(cov).view(-1, 1)
    out = {"loo_mu": mu_loo.ravel().numpy(), "loo_var": var_loo.ravel().numpy(),
           "loo_crps": float(crps(mu_loo, var_loo, y)), "loo_logs": float(logs(mu_loo, var_logs, y)),
           "nlml": 0.5 * n * LOG2PI + float(hl) + 0.5 * quad, "logdet": 2.0 * float(hl),
           "quad": quad, "pred_mu": mu.ravel().numpy(), "pred_var": var.ravel().numpy()}
    out.update(scores(mu, var, yt, y))
    return out


def host_info():
    """CPU model, the BLAS torch was built with, and its thread count (for cpu_baseline)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cfg = torch.__config__.show()
    blas = next((ln.split("=", 1)[1].strip().rstrip(",") for ln in cfg.replace(", ", "\n").splitlines()
                 if "BLAS_INFO" in ln), "unknown")
    lapack = next((ln.split("=", 1)[1].strip().rstrip(",") for ln in cfg.replace(", ", "\n").splitlines()
                   if "LAPACK_INFO" in ln), "unknown")
    return {"cpu_model": model, "blas": blas, "lapack": lapack, "torch": torch.__version__,
            "threads": torch.get_num_threads()}
