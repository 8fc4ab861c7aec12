"""Drop-in replacements for the reference scripts' helper functions.

Same names, argument order and meaning as the module-level helpers of
kin40k-FULL-compare.py (KF), KIN40K-COMPARE-ALL-FITC-20.py (K20) and
SIMPLE-DATA FULL-comapre.py (SD):

    ARD(x, xp, a, b)                                   KF:7-23
    rbf(x, xp, a, b)                                   SD:8-21
    chol_solve(B, A)                                   KF:25-29   -> A⁻¹B
    Q(a, u, b)                                         KF:32-39   (reads state.para_k / para_l)
    cal_mean_and_cov(k1, k2, k3, num, eye_num, data_y) KF:121-126 (reads state.sigma_noise_sq)
    spgp_cal_mean_and_cov(k1, Q1, Q2, k2, num_test, num_jitter, data_y)  K20:76-83
    crps(m, c, data_y) / logs(m, c, data_y)            KF:60-68 / KF:52-57
    trivial_loss(m, c, data_y, data_yp)                KF:110-119
    SMSE(m, data_y, data_yp)                           KF:128-134
    dss(m, c, shape1, data_y)                          KF:103-108
    ES(m, c, shape1, data_y, num_sim=300, beta=1)      KF:70-101  (draws: see ES)

The reference reads module globals ``para_k``, ``para_l``, ``sigma_noise_sq``
and ``dtype``; here they live on ``compat.state`` (settable attributes with the
same names) so the scripts' call sites work unchanged.  Inputs may be numpy
arrays or CPU torch tensors; outputs are float64 numpy arrays with the
reference's shapes (column vectors stay n×1, scalar objectives are floats).
All arithmetic runs through libgpscore.so on the GPU (Gram kernel, FP64 MFMA
GEMM, LDS Cholesky, score reductions).  ``cal_mean_and_cov`` returns the full
n*×n* covariance like the reference while n* <= FULL_COV_MAX; beyond that it
returns a ``DiagCov`` that only supports ``.diag()`` — the only use the
reference makes of it (KF:273, 372, 457; K20:277).
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np

from . import _lib
from ._lib import GPS_ARD, GPS_RBF, GPS_FULL, f64, ptr

FULL_COV_MAX = 4096
FITC_JITTER = 1e-3  # KF:36

state = SimpleNamespace(para_k=None, para_l=None, sigma_noise_sq=None, dtype="float64")


def _np(a):
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.asarray(a, dtype=np.float64)


def _scalar(a):
    return float(_np(a).ravel()[0])


def _ctx():
    return _lib.default_context()


def _gram(kind, x, xp, a, b):
    x, xp = f64(_np(x), 2), f64(_np(xp), 2)
    ell = np.ascontiguousarray(_np(b).ravel())
    out = np.empty((x.shape[0], xp.shape[0]))
    if out.size == 0:  # torch returns the empty n×m product for an empty side (KF:15-21)
        return out
    _ctx().call("gps_gram", kind, ptr(x), x.shape[0], ptr(xp), xp.shape[0], x.shape[1],
                _scalar(a), ptr(ell), ell.size, 0.0, GPS_FULL, ptr(out))
    return out


def ARD(x, xp, a, b):
    """sf2·exp(−½‖(x−x')/ℓ‖²), a = log sf2, b = log ℓ (scalar or 1×d). KF:7-23."""
    return _gram(GPS_ARD, x, xp, a, b)


def rbf(x, xp, a, b):
    """Isotropic SE with b = log ℓ² (SD:8-21)."""
    return _gram(GPS_RBF, x, xp, a, b)


def mm(A, B, transA=False, transB=False, alpha=1.0, beta=0.0, C=None):
    A, B = f64(_np(A), 2), f64(_np(B), 2)
    M = A.shape[1] if transA else A.shape[0]
    K = A.shape[0] if transA else A.shape[1]
    N = B.shape[0] if transB else B.shape[1]
    C = np.zeros((M, N)) if C is None else f64(C, 2).copy()
    _ctx().call("gps_gemm", int(transA), int(transB), M, N, K, alpha, ptr(A), A.shape[1], ptr(B),
                B.shape[1], beta, ptr(C), N)
    return C


def chol_solve(B, A):
    """A⁻¹B for SPD A (KF:25-29).  Raises NotPositiveDefinite (a RuntimeError) like torch.potrf."""
    A = f64(_np(A), 2)
    Bv = _np(B)
    vec = Bv.ndim == 1
    Bm = f64(Bv, 2)
    X = np.empty_like(Bm)
    _ctx().call("gps_potrs", A.shape[0], Bm.shape[1], ptr(A), A.shape[1], ptr(Bm), Bm.shape[1],
                ptr(X), X.shape[1])
    return X.ravel() if vec else X


def half_logdet(A):
    """potrf(A).diag().log().sum() (KF:332)."""
    A = f64(_np(A), 2).copy()
    ld = np.zeros(1)
    _ctx().call("gps_potrf", A.shape[0], ptr(A), A.shape[1], ptr(ld))
    return 0.5 * float(ld[0])


def diag_inv(A):
    """diag(chol_solve(I, A)) (KF:242) without forming A⁻¹."""
    A = f64(_np(A), 2)
    out = np.empty(A.shape[0])
    _ctx().call("gps_diag_inv", A.shape[0], ptr(A), A.shape[1], ptr(out))
    return out


def Q(a, u, b):
    """Nyström K_au (K_uu + 1e-3·I)⁻¹ K_ub with state.para_k / state.para_l (KF:32-39)."""
    K_au = ARD(a, u, state.para_k, state.para_l)
    K_uu = ARD(u, u, state.para_k, state.para_l)
    K_uu_j = K_uu + FITC_JITTER * np.eye(K_uu.shape[0])
    K_ub = ARD(u, b, state.para_k, state.para_l)
    return mm(K_au, chol_solve(K_ub, K_uu_j))


class DiagCov:
    """Predictive covariance carried as its diagonal only (n* > FULL_COV_MAX)."""

    def __init__(self, d):
        self._d = np.asarray(d)

    def diag(self):
        return self._d

    @property
    def shape(self):
        return (self._d.size, self._d.size)


def cal_mean_and_cov(k1, k2, k3, num, eye_num, data_y):
    """Full-GP predictive (KF:121-126): mean K*f A⁻¹y, cov σ²I + K** − K*f A⁻¹ Kf*."""
    s2 = _scalar(state.sigma_noise_sq)
    k1, k2, k3 = f64(_np(k1), 2), f64(_np(k2), 2), f64(_np(k3), 2)
    y = f64(_np(data_y), 2)
    jk = k2 + s2 * np.eye(int(eye_num))
    mean = mm(k1, chol_solve(y, jk))
    W = chol_solve(k1.T, jk)
    num = int(num)
    if num <= FULL_COV_MAX:
        return mean, mm(k1, W, alpha=-1.0, beta=1.0, C=k3 + s2 * np.eye(num))
    d = np.empty(num)
    for r0 in range(0, num, FULL_COV_MAX):
        r1 = min(num, r0 + FULL_COV_MAX)
        blk = mm(k1[r0:r1], np.ascontiguousarray(W[:, r0:r1]), alpha=-1.0, beta=1.0,
                 C=k3[r0:r1, r0:r1] + s2 * np.eye(r1 - r0))
        d[r0:r1] = np.diag(blk)
    return mean, DiagCov(d)


def spgp_cal_mean_and_cov(k1, Q1, Q2, k2, num_test, num_jitter, data_y):
    """FITC predictive (K20:76-83) with G = diag(K_ff − Q_ff + σ²I)."""
    s2 = _scalar(state.sigma_noise_sq)
    k1, Q1, Q2, k2 = (f64(_np(a), 2) for a in (k1, Q1, Q2, k2))
    y = f64(_np(data_y), 2)
    G = np.diag(np.diag(k1 - Q1 + s2 * np.eye(int(num_jitter))))
    big = Q1 + G
    mean = mm(Q2, chol_solve(y, big))
    cov = mm(Q2, chol_solve(Q2.T, big), alpha=-1.0, beta=1.0, C=k2 + s2 * np.eye(int(num_test)))
    return mean, cov


def _scores(m, c, y, yp=None):
    m, c, y = (f64(_np(a)).ravel() for a in (m, c, y))
    if yp is None:
        mu0, v0 = 0.0, 1.0
    else:
        ypv = f64(_np(yp)).ravel()
        mu0, v0 = float(ypv.mean()), float(ypv.var(ddof=1))
    if y.size == 0:  # torch.mean over no points is NaN (KF:57, KF:68), not an error
        return np.full(6, np.nan)
    out = np.zeros(6)
    _ctx().call("gps_scores", ptr(m), ptr(c), ptr(y), y.size, mu0, v0, ptr(out))
    return out


def crps(m, c, data_y):
    """Mean Gaussian CRPS, c = variance (KF:60-68)."""
    return float(_scores(m, c, data_y)[0])


def logs(m, c, data_y):
    """Mean negative log predictive density (KF:52-57)."""
    return float(_scores(m, c, data_y)[1])


def trivial_loss(m, c, data_y, data_yp):
    """MSLL against N(mean(y_train), unbiased var(y_train)) (KF:110-119)."""
    return float(_scores(m, c, data_y, data_yp)[2])


def SMSE(m, data_y, data_yp):
    """MSE / MSE of the train-mean predictor (KF:128-134)."""
    m = f64(_np(m)).ravel()
    return float(_scores(m, np.ones_like(m), data_y, data_yp)[3])


def dss(m, c, shape1, data_y):
    """Dawid–Sebastiani score of N(m, c) at data_y (KF:103-108; K20:106-111 inverts c instead of
    solving, the same number): ½·shape1·log2π + ½log|c| + ½(y − m)ᵀc⁻¹(y − m)."""
    C = f64(_np(c), 2)
    r = (f64(_np(data_y)).ravel() - f64(_np(m)).ravel()).reshape(-1, 1)
    quad = float(mm(r, chol_solve(r, C), transA=True)[0, 0])
    return 0.5 * int(shape1) * LOG2PI + half_logdet(C) + 0.5 * quad


def ES(m, c, shape1, data_y, num_sim=300, beta=1, draws=None, rng=None):
    """Energy score of N(m, c) at data_y from num_sim draws (KF:70-101):
    (1/S)Σ_i ‖z_i − (m − y)‖^β − Σ_ij ‖z_i − z'_j‖^β / (2S(S−1)),  z = ξc^½, z' = ξ'c^½.
    ``draws`` (2·num_sim·shape1 values: ξ then ξ', row-major) fixes ξ, ξ'; the reference
    draws them with torch.randn on every call — here from ``rng`` (numpy) when not given."""
    C = f64(_np(c), 2)
    b = C.shape[0]
    if int(shape1) != b:
        raise ValueError("shape1 must be c's order (the draws are num_sim × shape1, KF:79)")
    mv, yv = f64(_np(m)).ravel(), f64(_np(data_y)).ravel()
    if draws is None:
        draws = np.random.default_rng(rng).standard_normal(2 * int(num_sim) * b)
    draws = f64(draws).ravel()
    if draws.size != 2 * int(num_sim) * b:
        raise ValueError("draws must hold 2·num_sim·shape1 values")
    out = np.zeros(1)
    _ctx().call("gps_energy_score", ptr(mv), ptr(C), b, ptr(yv), int(num_sim), float(beta),
                ptr(draws), ptr(out))
    return float(out[0])


LOG2PI = math.log(2.0 * math.pi)
