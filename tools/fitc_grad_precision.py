"""FITC gradient conditioning study: the round-3 explicit-inverse
formulation vs the whitened one, (a) moved by input perturbations of 1e-15 ... 1e-9 (relative),
(b) against an 80-bit (numpy longdouble) evaluation of the whitened formula.  CPU only.
Usage: python tools/fitc_grad_precision.py > profiles/r4_fitc_grad_conditioning.txt"""
import sys, math, numpy as np, mpmath
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import gp_oracle as O
from conftest import nrel
LD = np.longdouble
mpmath.mp.prec = 80

def chol(A):
    A = A.copy(); m = A.shape[0]; L = np.zeros_like(A)
    for j in range(m):
        s = A[j, j] - np.sum(L[j, :j] ** 2)
        L[j, j] = np.sqrt(s)
        L[j+1:, j] = (A[j+1:, j] - L[j+1:, :j] @ L[j, :j]) / L[j, j]
    return L

def trinv(L):
    m = L.shape[0]; X = np.zeros_like(L)
    for i in range(m):
        X[i, i] = 1 / L[i, i]
        for j in range(i):
            X[i, j] = -np.sum(L[i, j:i] * X[j:i, j]) / L[i, i]
    return X

def gram(X, Z, sf2, ell):
    D = np.zeros((X.shape[0], Z.shape[0]), dtype=X.dtype)
    for k in range(X.shape[1]):
        D += ((X[:, k:k+1] - Z[None, :, k]) / ell[k]) ** 2
    return sf2 * np.exp(-0.5 * D)

def erf(x):
    return np.array([LD(str(mpmath.erf(mpmath.mpf(str(v))))) for v in x], dtype=LD) if x.dtype == LD else O._erf(x)

def score_derivs(obj, m, c, y):
    n = y.size
    if obj == "loo_crps":
        s = np.sqrt(c); z = (y - m) / s
        cdf = (1 + erf(z / np.sqrt(c.dtype.type(2)))) / 2
        pi = c.dtype.type(np.pi) if c.dtype != LD else LD("3.14159265358979323846264338327950288")
        pdf = np.exp(-z * z / 2) / np.sqrt(2 * pi)
        return (1 - 2 * cdf) / n, (2 * pdf - 1 / np.sqrt(pi)) / (2 * s * n)
    r = y - m
    return -r / (c * n), (1 / (2 * c) - r * r / (2 * c * c)) / n

def fitc_grad_explicit(X, y, Z, log_sf2, log_ell, log_sn2, obj, dt=np.float64):
    """round 3's formulation: explicit Km⁻¹ = Lm⁻ᵀLm⁻¹ and B⁻¹ = Lb⁻ᵀLb⁻¹ in the n×m products"""
    X, Z, y = X.astype(dt), Z.astype(dt), y.astype(dt)
    n, nd = X.shape; m = Z.shape[0]
    ell = np.exp(np.asarray(log_ell, dt) * np.ones(nd, dt)); sf2 = np.exp(dt(log_sf2)); sn2 = np.exp(dt(log_sn2))
    Kzz = gram(Z, Z, sf2, ell); Kmm = Kzz + dt(1e-3) * np.eye(m, dtype=dt)
    Lm = chol(Kmm); Lmi = trinv(Lm)
    K = gram(X, Z, sf2, ell)
    V = K @ Lmi.T
    lam = sf2 - np.sum(V * V, 1) + sn2
    B = Kmm + K.T @ (K / lam[:, None]); bb = (K / lam[:, None]).T @ y
    Lb = chol(B); Lbi = trinv(Lb)
    c = Lbi.T @ (Lbi @ bb)
    Binv = Lbi.T @ Lbi; Kminv = Lmi.T @ Lmi
    KB = K @ Binv; r = np.sum(KB * K, 1)
    dinv = 1 / lam - r / lam ** 2
    alpha = (y - K @ c) / lam
    mu, var = y - alpha / dinv, 1 / dinv
    if obj == "nlml":
        a, v, h = dt(0.5), alpha / 2, np.zeros(n, dt)
    else:
        g_mu, g_c = score_derivs(obj, mu, var, y)
        u = -g_mu / dinv; h = (g_mu * alpha - g_c) / (dinv * dinv)
        v = u / lam - (KB @ (K.T @ (u / lam))) / lam; a = dt(0)
    S2 = K.T @ (K * (h / lam ** 2)[:, None]); N = Binv @ S2 @ Binv; KN = K @ N
    q = np.sum(KN * K, 1)
    Md = a * dinv - v * alpha - (h / lam ** 2 - 2 * h * r / lam ** 3 + q / lam ** 2)
    w_hat = Kminv @ (K.T @ v)
    GK = ((2 * (a / lam - h / lam ** 2))[:, None] * KB + (2 / lam)[:, None] * KN
          - (2 * Md)[:, None] * (K @ Kminv) - np.outer(v, c) - np.outer(alpha, w_hat))
    KmD = Kminv @ (K.T @ (K * Md[:, None])) @ Kminv
    GKm = -a * (Kminv - Binv) + (np.outer(w_hat, c) + np.outer(c, w_hat)) / 2 + N + KmD
    GKK, GmK = GK * K, GKm * Kzz
    gl = np.empty(nd, dt); gZ = np.empty((m, nd), dt)
    for k in range(nd):
        dxz = (X[:, k:k+1] - Z[None, :, k]) / ell[k]; dzz = (Z[:, k:k+1] - Z[None, :, k]) / ell[k]
        gl[k] = np.sum(GKK * dxz * dxz) + np.sum(GmK * dzz * dzz)
        gZ[:, k] = (np.sum(GKK * dxz, 0) - 2 * np.sum(GmK * dzz, 1)) / ell[k]
    g = np.concatenate([[np.sum(GKK) + np.sum(GmK) + sf2 * np.sum(Md)], gl, [sn2 * np.sum(Md)]])
    return g, gZ, dict(GK=GK, GKm=GKm, Md=Md, v=v, alpha=alpha, w_hat=w_hat, c=c, KB=KB, KN=KN, Kminv=Kminv, K=K)


def fitc_grad_w(X, y, Z, log_sf2, log_ell, log_sn2, obj, dt=np.float64):
    """whitened: V = K Lm^-T, U = K Lb^-T; no explicit Km^-1 / B^-1"""
    X, Z, y = X.astype(dt), Z.astype(dt), y.astype(dt)
    n, nd = X.shape; m = Z.shape[0]
    ell = np.exp(np.asarray(log_ell, dt) * np.ones(nd, dt)); sf2 = np.exp(dt(log_sf2)); sn2 = np.exp(dt(log_sn2))
    Kzz = gram(Z, Z, sf2, ell); Kmm = Kzz + dt(1e-3) * np.eye(m, dtype=dt)
    Lm = chol(Kmm); Lmi = trinv(Lm)
    K = gram(X, Z, sf2, ell)
    V = K @ Lmi.T
    lam = sf2 - np.sum(V * V, 1) + sn2
    B = Kmm + K.T @ (K / lam[:, None]); bb = (K / lam[:, None]).T @ y
    Lb = chol(B); Lbi = trinv(Lb)
    c = Lbi.T @ (Lbi @ bb)
    U = K @ Lbi.T
    r = np.sum(U * U, 1)
    dinv = 1 / lam - r / lam ** 2
    alpha = (y - K @ c) / lam
    mu, var = y - alpha / dinv, 1 / dinv
    if obj == "nlml":
        a, v, h = dt(0.5), alpha / 2, np.zeros(n, dt)
    else:
        g_mu, g_c = score_derivs(obj, mu, var, y)
        u = -g_mu / dinv; h = (g_mu * alpha - g_c) / (dinv * dinv)
        v = u / lam - (U @ (U.T @ (u / lam))) / lam; a = dt(0)
    D = h / lam ** 2
    P = U.T @ (U * D[:, None])
    UP = U @ P
    q = np.sum(UP * U, 1)
    Md = a * dinv - v * alpha - (h / lam ** 2 - 2 * h * r / lam ** 3 + q / lam ** 2)
    w_hat = Lmi.T @ (V.T @ v)
    Y = (2 * (a / lam - h / lam ** 2))[:, None] * U + (2 / lam)[:, None] * UP
    GK = Y @ Lbi - (2 * Md)[:, None] * (V @ Lmi) - np.outer(v, c) - np.outer(alpha, w_hat)
    KmD = Lmi.T @ (V.T @ (V * Md[:, None])) @ Lmi
    N = Lbi.T @ P @ Lbi
    GKm = -a * (Lmi.T @ Lmi - Lbi.T @ Lbi) + (np.outer(w_hat, c) + np.outer(c, w_hat)) / 2 + N + KmD
    GKK, GmK = GK * K, GKm * Kzz
    gl = np.empty(nd, dt); gZ = np.empty((m, nd), dt)
    for k in range(nd):
        dxz = (X[:, k:k+1] - Z[None, :, k]) / ell[k]; dzz = (Z[:, k:k+1] - Z[None, :, k]) / ell[k]
        gl[k] = np.sum(GKK * dxz * dxz) + np.sum(GmK * dzz * dzz)
        gZ[:, k] = (np.sum(GKK * dxz, 0) - 2 * np.sum(GmK * dzz, 1)) / ell[k]
    g = np.concatenate([[np.sum(GKK) + np.sum(GmK) + sf2 * np.sum(Md)], gl, [sn2 * np.sum(Md)]])
    return g, gZ, dict(GK=GK, GKm=GKm, Md=Md, v=v, N=N, KmD=KmD)


def main():
    rng = np.random.default_rng(1000 + 37 + 3)   # tests/test_gpu_fitc_grad.py ill-conditioned case
    n, m, d = 1000, 37, 3
    X = rng.standard_normal((n, d)); y = np.sin(X.sum(1)) + 0.1 * rng.standard_normal(n)
    Z = X[rng.choice(n, m, replace=False)] + 0.05 * rng.standard_normal((m, d))
    th = (0.1, np.log(np.linspace(1.0, 3.0, d)), np.log(0.05))
    Kmm, _, _ = O.fitc_shared(Z, *th[:2])
    cond = np.linalg.cond(Kmm)
    kappa = cond * (np.exp(0.1) + 0.05) / 0.05
    print("case n=%d m=%d d=%d  cond(Kmm)=%.3g  kappa=%.3g  kappa*eps=%.2e" % (n, m, d, cond, kappa, kappa * 2.22e-16))
    for obj in ("nlml", "loo_crps", "loo_logs"):
        gt, zt, _ = fitc_grad_w(X, y, Z, *th, obj, LD)
        gt, zt = gt.astype(float), zt.astype(float)
        for name, f in (("explicit", fitc_grad_explicit), ("whitened", fitc_grad_w)):
            g0, z0, _ = f(X, y, Z, *th, obj)
            print("%-8s %-9s vs 80-bit: grad %.2e  grad_Z %.2e" % (obj, name, nrel(g0, gt), nrel(z0, zt)))
            for dl in (1e-15, 1e-13, 1e-11, 1e-9):
                r = np.random.default_rng(1)
                g, z, _ = f(X * (1 + dl * r.standard_normal(X.shape)), y, Z * (1 + dl * r.standard_normal(Z.shape)), *th, obj)
                print("   perturbation %.0e: grad moves %.2e  grad_Z %.2e" % (dl, nrel(g, g0), nrel(z, z0)))


if __name__ == "__main__":
    main()
