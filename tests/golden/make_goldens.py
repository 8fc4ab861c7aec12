"""Generate the golden input/output vectors that pin the oracle and the HIP path.

This script runs ONLY in the build container, where the read-only reference tree
is mounted at /root/reference.  It never copies reference source into this repo:
at run time it parses the reference scripts with ``ast``, extracts the top-level
helper ``def``s (ARD, rbf, chol_solve, Q, cal_mean_and_cov,
spgp_cal_mean_and_cov, crps, logs, trivial_loss, SMSE), and executes them in a
private namespace with a two-line compatibility shim for the torch-0.4 era API
the reference targets:

* ``torch.potrf(A)``  -> ``torch.linalg.cholesky(A, upper=True)`` (0.4 default: upper)
* ``torch.gesv(B, A)`` -> ``(torch.linalg.solve(A, B), None)``   (LU with pivoting,
  the same semantics as LAPACK ?gesv)

Everything runs in float64 (``torch.set_default_dtype(torch.float64)`` and
``dtype = torch.DoubleTensor``) so the goldens are the reference algorithm at
fp64.  The per-iteration objective bodies of the reference are inline script
code, not defs; they are composed here from the extracted defs exactly as the
reference writes them, with the file:line of each body cited next to it.

Only data leaves this script: ``tests/golden/*.npz`` (inputs + expected outputs).

Usage:  python tests/golden/make_goldens.py
"""
from __future__ import annotations

import ast
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

# which file each helper is taken from (all helpers are AST-identical across the
# four scripts; rbf exists only in SD/SF)
SOURCES = {
    "kin40k-FULL-compare.py": ["ARD", "chol_solve", "Q", "crps", "logs",
                               "trivial_loss", "cal_mean_and_cov", "SMSE", "dss", "ES"],
    "KIN40K-COMPARE-ALL-FITC-20.py": ["spgp_cal_mean_and_cov"],
    "SIMPLE-DATA FULL-comapre.py": ["rbf"],
}


class _TorchShim(types.ModuleType):
    """torch with the two removed 0.4-era entry points restored."""

    def __init__(self):
        super().__init__("torch")

    def __getattr__(self, name):
        return getattr(torch, name)

    @staticmethod
    def potrf(A, upper=True):
        return torch.linalg.cholesky(A, upper=upper)

    @staticmethod
    def gesv(B, A):
        return torch.linalg.solve(A, B), None


def load_reference_defs():
    if not os.path.isdir(REF):
        raise SystemExit(f"{REF} not present: goldens can only be regenerated in the build container")
    ns = {"torch": _TorchShim(), "math": math, "np": np,
          "dtype": torch.DoubleTensor}
    for fname, names in SOURCES.items():
        with open(os.path.join(REF, fname), "r", encoding="utf-8", errors="replace") as fh:
            tree = ast.parse(fh.read().replace("\r\n", "\n"))
        found = {}
        for node in tree.body:
            if isinstance(node, ast.FunctionDef) and node.name in names and node.name not in found:
                found[node.name] = node
        missing = set(names) - set(found)
        if missing:
            raise SystemExit(f"defs {missing} not found in {fname}")
        mod = ast.Module(body=list(found.values()), type_ignores=[])
        exec(compile(mod, f"<reference:{fname}>", "exec"), ns)
    # K20 has its own dss (cov_term.inverse() instead of chol_solve, K20:106-111): load it
    # under another name for the FITC block-LOO bodies
    for fname, name, alias in (("KIN40K-COMPARE-ALL-FITC-20.py", "dss", "dss_k20"),):
        with open(os.path.join(REF, fname), "r", encoding="utf-8", errors="replace") as fh:
            tree = ast.parse(fh.read().replace("\r\n", "\n"))
        node = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name)
        sub = {"torch": ns["torch"], "math": math, "np": np, "chol_solve": ns["chol_solve"]}
        exec(compile(ast.Module(body=[node], type_ignores=[]), f"<reference:{fname}>", "exec"), sub)
        ns[alias] = sub[name]
    return ns


def T(a):
    return torch.as_tensor(np.asarray(a, dtype=np.float64))


def full_case(ns, X, y, Xt, yt, log_sf2, log_ell, log_sn2, kern="ARD"):
    """Full GP objectives + predictive + scores, composed as the reference does."""
    K = ns[kern]
    ns["dtype"] = torch.DoubleTensor
    para_k = T([log_sf2])
    para_l = T(np.atleast_1d(log_ell)).view(1, -1) if kern == "ARD" else T([log_ell])
    para_noise = T([log_sn2])
    ns["para_k"], ns["para_l"] = para_k, para_l
    train_x, train_y, test_x, test_y = T(X), T(y).view(-1, 1), T(Xt), T(yt).view(-1, 1)
    n, nt = train_x.shape[0], test_x.shape[0]
    out = {}
    with torch.no_grad():
        sigma_noise_sq = torch.exp(para_noise)            # KF:239
        ns["sigma_noise_sq"] = sigma_noise_sq
        k_ff = K(train_x, train_x, para_k, para_l)          # KF:240
        big_k = k_ff + sigma_noise_sq * torch.eye(n)        # KF:241
        k_ii_diag = torch.diag(ns["chol_solve"](torch.eye(n), big_k)).view(n, 1)  # KF:242
        mean_term = train_y - ns["chol_solve"](train_y, big_k) / k_ii_diag       # KF:243
        cov_term = 1 / k_ii_diag                                                 # KF:244
        out["loo_mu"] = mean_term.view(-1).numpy()
        out["loo_var"] = cov_term.view(-1).numpy()
        out["loo_crps"] = ns["crps"](mean_term, cov_term, train_y).item()      # KF:245
        out["loo_logs"] = ns["logs"](mean_term, cov_term, train_y).item()      # KF:424
        # NLML body, KF:329-334
        inverse_term_ml = k_ff + torch.eye(n) * sigma_noise_sq
        half_log_det = torch.linalg.cholesky(inverse_term_ml, upper=True).diag().log().sum()
        quad = (train_y.transpose(0, 1)).mm(ns["chol_solve"](train_y, inverse_term_ml))
        nlml = torch.tensor([0.5 * n * (np.log(2 * np.pi))]) + half_log_det + 0.5 * quad
        out["nlml"] = nlml.item()
        out["logdet"] = 2.0 * half_log_det.item()
        out["quad"] = quad.item()
        # predict (KF:267-273 via cal_mean_and_cov) + score (KF:276-292)
        k_star_f = K(test_x, train_x, para_k, para_l)
        k_ss = K(test_x, test_x, para_k, para_l)
        mu, cov = ns["cal_mean_and_cov"](k_star_f, k_ff, k_ss, nt, eye_num=n, data_y=train_y)
        var = cov.diag().view(nt, 1)
        out.update(score_block(ns, mu, var, test_y, train_y))
        out["pred_mu"] = mu.view(-1).numpy()
        out["pred_var"] = var.view(-1).numpy()
    return out


def score_block(ns, mu, var, test_y, train_y):
    """KF:276-292 (MSE, SMSE, LogS, CRPS, MSLL, ±2σ coverage)."""
    up = mu + 2 * var ** 0.5
    low = mu - 2 * var ** 0.5
    cov_frac = np.multiply(((up - test_y) > 0).numpy(), ((test_y - low) > 0).numpy()).mean()
    return {
        "test_mse": ((mu - test_y) ** 2).mean().item(),
        "test_smse": ns["SMSE"](mu, test_y, train_y).item(),
        "test_logs": ns["logs"](mu, var, test_y).item(),
        "test_crps": ns["crps"](mu, var, test_y).item(),
        "test_msll": ns["trivial_loss"](mu, var, test_y, train_y).item(),
        "test_cover": float(cov_frac),
    }


def fitc_case(ns, X, y, Xt, yt, Z, log_sf2, log_ell, log_sn2):
    """FITC objectives (K20:222-234, 329-340, 434-447) + predictive (K20:270-296)."""
    para_k = T([log_sf2])
    para_l = T(np.atleast_1d(log_ell)).view(1, -1)
    para_noise = T([log_sn2])
    ns["para_k"], ns["para_l"], ns["dtype"] = para_k, para_l, torch.DoubleTensor
    train_x, train_y, test_x, test_y = T(X), T(y).view(-1, 1), T(Xt), T(yt).view(-1, 1)
    inducing_x = T(Z)
    n, nt = train_x.shape[0], test_x.shape[0]
    ARD, Qf, chol_solve = ns["ARD"], ns["Q"], ns["chol_solve"]
    out = {}
    with torch.no_grad():
        sigma_noise_sq = torch.exp(para_noise)
        ns["sigma_noise_sq"] = sigma_noise_sq
        k_ff = ARD(train_x, train_x, para_k, para_l)                       # K20:223
        Q_ff = Qf(train_x, inducing_x, train_x)                           # K20:224
        G = (torch.diag(k_ff - Q_ff + sigma_noise_sq * torch.eye(n)) * torch.eye(n))  # K20:225-228
        big_Q = Q_ff + G                                                   # K20:229
        Q_ii_diag = torch.diag(chol_solve(torch.eye(n), big_Q)).view(n, 1) # K20:230
        mean_term = train_y - chol_solve(train_y, big_Q) / Q_ii_diag       # K20:231
        cov_term = 1 / Q_ii_diag                                           # K20:232
        out["loo_mu"] = mean_term.view(-1).numpy()
        out["loo_var"] = cov_term.view(-1).numpy()
        out["loo_crps"] = ns["crps"](mean_term, cov_term, train_y).item()  # K20:234
        # LogS variant, K20:442-447
        small_Q = torch.diag(big_Q).view(n, 1)
        small_k = torch.diag(k_ff).view(n, 1)
        cov_logs = 1 / Q_ii_diag + sigma_noise_sq - small_Q + small_k
        out["loo_logs"] = ns["logs"](mean_term, cov_logs, train_y).item()
        # NLML, K20:332-340
        G2 = torch.eye(n) * torch.diag(k_ff - Q_ff + sigma_noise_sq * torch.eye(n))
        inverse_term_ml = Q_ff + G2
        half_log_det = torch.linalg.cholesky(inverse_term_ml, upper=True).diag().log().sum()
        quad = (train_y.transpose(0, 1)).mm(chol_solve(train_y, inverse_term_ml))
        nlml = torch.tensor([0.5 * n * (np.log(2 * np.pi))]) + half_log_det + 0.5 * quad
        out["nlml"] = nlml.item()
        out["logdet"] = 2.0 * half_log_det.item()
        out["quad"] = quad.item()
        # predict, K20:270-277
        k_ss = ARD(test_x, test_x, para_k, para_l)
        Q_sf = Qf(test_x, inducing_x, train_x)
        mu, cov = ns["spgp_cal_mean_and_cov"](k_ff, Q_ff, Q_sf, k_ss, nt, n, train_y)
        var = cov.diag().view(-1, 1)
        out.update(score_block(ns, mu, var, test_y, train_y))
        out["pred_mu"] = mu.view(-1).numpy()
        out["pred_var"] = var.view(-1).numpy()
    return out


def grads_full(ns, X, y, log_sf2, log_ell, log_sn2, kern="ARD"):
    """Autograd gradients of the three full-GP objectives (KF:252, 339, 428): for next-1.
    kern = "ARD" (b = log ℓ, scalar or per-dimension) or "rbf" (b = log ℓ², SD:8-21)."""
    res = {}
    for obj in ("loo_crps", "nlml", "loo_logs"):
        para_k = T([log_sf2]).requires_grad_(True)
        para_l = T(np.atleast_1d(log_ell)).view(1, -1).clone().requires_grad_(True)
        para_noise = T([log_sn2]).requires_grad_(True)
        train_x, train_y = T(X), T(y).view(-1, 1)
        n = train_x.shape[0]
        sigma_noise_sq = torch.exp(para_noise)
        k_ff = ns[kern](train_x, train_x, para_k, para_l)
        big_k = k_ff + sigma_noise_sq * torch.eye(n)
        if obj == "nlml":
            hl = torch.linalg.cholesky(big_k, upper=True).diag().log().sum()
            val = 0.5 * n * np.log(2 * np.pi) + hl + 0.5 * (train_y.t()).mm(ns["chol_solve"](train_y, big_k))
        else:
            kii = torch.diag(ns["chol_solve"](torch.eye(n), big_k)).view(n, 1)
            mt = train_y - ns["chol_solve"](train_y, big_k) / kii
            val = (ns["crps"] if obj == "loo_crps" else ns["logs"])(mt, 1 / kii, train_y)
        val.sum().backward()
        res[f"grad_{obj}"] = np.concatenate([para_k.grad.numpy().ravel(),
                                             para_l.grad.numpy().ravel(),
                                             para_noise.grad.numpy().ravel()])
    return res


def grads_fitc(ns, X, y, Z, log_sf2, log_ell, log_sn2):
    """Autograd gradients of the three FITC objectives w.r.t. (para_k, para_l, para_noise)
    and inducing_x — the `.backward()` at K20:236 (LOO-CRPS, body K20:222-234), K20:344
    (NLML, body K20:329-340) and K20:452 (LOO-LogS, body K20:434-447).  Inducing points are
    trained parameters in the reference (K20:247)."""
    res = {}
    for obj in ("loo_crps", "nlml", "loo_logs"):
        para_k = T([log_sf2]).requires_grad_(True)
        para_l = T(np.atleast_1d(log_ell)).view(1, -1).clone().requires_grad_(True)
        para_noise = T([log_sn2]).requires_grad_(True)
        inducing_x = T(Z).clone().requires_grad_(True)
        ns["para_k"], ns["para_l"], ns["dtype"] = para_k, para_l, torch.DoubleTensor
        train_x, train_y = T(X), T(y).view(-1, 1)
        n = train_x.shape[0]
        ARD, Qf, chol_solve = ns["ARD"], ns["Q"], ns["chol_solve"]
        sigma_noise_sq = torch.exp(para_noise)
        k_ff = ARD(train_x, train_x, para_k, para_l)
        Q_ff = Qf(train_x, inducing_x, train_x)
        G = torch.diag(k_ff - Q_ff + sigma_noise_sq * torch.eye(n)) * torch.eye(n)
        big_Q = Q_ff + G
        if obj == "nlml":                                                  # K20:337-340
            hl = torch.linalg.cholesky(big_Q, upper=True).diag().log().sum()
            val = (torch.tensor([0.5 * n * np.log(2 * np.pi)]) + hl
                   + 0.5 * (train_y.transpose(0, 1)).mm(chol_solve(train_y, big_Q)))
        else:
            Q_ii_diag = torch.diag(chol_solve(torch.eye(n), big_Q)).view(n, 1)
            mean_term = train_y - chol_solve(train_y, big_Q) / Q_ii_diag
            if obj == "loo_crps":                                          # K20:230-234
                val = ns["crps"](mean_term, 1 / Q_ii_diag, train_y)
            else:                                                          # K20:441-447
                small_Q = torch.diag(big_Q).view(n, 1)
                small_k = torch.diag(k_ff).view(n, 1)
                cov_term = 1 / Q_ii_diag + sigma_noise_sq - small_Q + small_k
                val = ns["logs"](mean_term, cov_term, train_y)
        val.sum().backward()
        res[f"grad_{obj}"] = np.concatenate([para_k.grad.numpy().ravel(),
                                             para_l.grad.numpy().ravel(),
                                             para_noise.grad.numpy().ravel()])
        res[f"gradZ_{obj}"] = inducing_x.grad.numpy().copy()
        res[f"value_{obj}"] = float(val.detach().sum())
    return res


def block_loo_case(ns, X, y, log_sf2, log_ell, log_sn2, Z=None, with_grad=True):
    """4-fold block-LOO objectives composed exactly as the scripts write them: full GP DSS
    (KF:494-543, dss KF:103-108), FITC DSS (K20:536-587, dss K20:106-111) and FITC KC
    (K20:669-720); "kc" on the full GP applies the K20:682-714 KC body to big_k.  Returns
    values and autograd gradients (θ; and inducing_x for FITC)."""
    out = {}
    for obj in ("dss", "kc"):
        para_k = T([log_sf2]).requires_grad_(True)
        para_l = T(np.atleast_1d(log_ell)).view(1, -1).clone().requires_grad_(True)
        para_noise = T([log_sn2]).requires_grad_(True)
        ns["para_k"], ns["para_l"], ns["dtype"] = para_k, para_l, torch.DoubleTensor
        train_x, train_y = T(X), T(y).view(-1, 1)
        num_train = train_x.shape[0]
        chol_solve, crps = ns["chol_solve"], ns["crps"]
        sigma_noise_sq = torch.exp(para_noise)
        k_ff = ns["ARD"](train_x, train_x, para_k, para_l)
        fold_k = 4
        index1 = int(num_train / fold_k)
        index2 = int(2 * num_train / fold_k)
        index3 = int(3 * num_train / fold_k)
        if Z is None:
            big = k_ff + sigma_noise_sq * torch.eye(num_train)
            dss = ns["dss"]
        else:
            inducing_x = T(Z).clone().requires_grad_(True)
            Q_ff = ns["Q"](train_x, inducing_x, train_x)
            G = (torch.diag(k_ff - Q_ff + sigma_noise_sq * torch.eye(num_train))
                 * torch.eye(num_train)).type(torch.DoubleTensor)
            big = Q_ff + G
            dss = ns["dss_k20"]
        inv_ij = chol_solve(torch.eye(num_train), big)
        sl = [slice(0, index1), slice(index1, index2), slice(index2, index3),
              slice(index3, num_train)]
        inv_y = chol_solve(train_y, big)
        tot = 0
        for s_ in sl:
            kb = inv_ij[s_, s_]
            yb = train_y[s_]
            m = yb - chol_solve(torch.eye(index1), kb).mm(inv_y[s_])
            if obj == "dss":
                cov = chol_solve(torch.eye(index1), kb)
                tot = tot + dss(m, cov, index1, yb)
            else:
                cov = torch.diag(chol_solve(torch.eye(index1), kb)).view(index1, 1)
                tot = tot + crps(m, cov, yb)
        val = tot.mean()
        if with_grad:
            val.backward()
            out[f"grad_{obj}"] = np.concatenate([para_k.grad.numpy().ravel(),
                                                 para_l.grad.numpy().ravel(),
                                                 para_noise.grad.numpy().ravel()])
            if Z is not None:
                out[f"gradZ_{obj}"] = inducing_x.grad.numpy().copy()
        out[f"value_{obj}"] = float(val.detach())
    return out


def es_case(ns, X, y, log_sf2, log_ell, log_sn2, num_sim, seed):
    """4-fold block-LOO energy score composed as the ES loop writes it (KF:615-663; ES
    KF:70-101 through the extracted def): value, autograd gradient, and the standard-normal
    draws its torch.randn calls consumed — the same seed replayed, fold by fold ξ then ξ'
    (KF:79-80), in the layout the C-ABI takes."""
    para_k = T([log_sf2]).requires_grad_(True)
    para_l = T(np.atleast_1d(log_ell)).view(1, -1).clone().requires_grad_(True)
    para_noise = T([log_sn2]).requires_grad_(True)
    ns["para_k"], ns["para_l"], ns["dtype"] = para_k, para_l, torch.DoubleTensor
    train_x, train_y = T(X), T(y).view(-1, 1)
    num_train = train_x.shape[0]
    chol_solve = ns["chol_solve"]
    sigma_noise_sq = torch.exp(para_noise)                                    # KF:618
    k_ff = ns["ARD"](train_x, train_x, para_k, para_l)                        # KF:619
    fold_k = 4
    index1 = int(num_train / fold_k)
    index2 = int(2 * num_train / fold_k)
    index3 = int(3 * num_train / fold_k)
    big_k = k_ff + sigma_noise_sq * torch.eye(num_train)                      # KF:625
    k_inv_i_j = chol_solve(torch.eye(num_train), big_k)                       # KF:626
    k_inv_y = chol_solve(train_y, big_k)                                       # KF:638
    sl = [slice(0, index1), slice(index1, index2), slice(index2, index3),
          slice(index3, num_train)]
    torch.manual_seed(seed)
    tot = 0
    for s_ in sl:
        kb = k_inv_i_j[s_, s_]
        yb = train_y[s_]
        m = yb - chol_solve(torch.eye(index1), kb).mm(k_inv_y[s_])             # KF:640-643
        cov = chol_solve(torch.eye(index1), kb)                                # KF:646-649
        tot = tot + ns["ES"](m, cov, index1, yb, num_sim)                      # KF:652-655
    val = tot.mean()                                                           # KF:657
    val.backward()                                                             # KF:663
    torch.manual_seed(seed)
    draws = np.concatenate([torch.randn(num_sim, index1).numpy().ravel() for _ in range(2 * fold_k)])
    return {"value_es": float(val.detach()),
            "grad_es": np.concatenate([para_k.grad.numpy().ravel(), para_l.grad.numpy().ravel(),
                                       para_noise.grad.numpy().ravel()]),
            "draws_es": draws, "num_sim": num_sim}


def surface_case(ns, x, y, ell_grid, sd_grid):
    """contour-plot.R's four objectives (CP.R:43-85) on a grid, composed from the Python
    reference defs with CP.R's parameterisation: the reference rbf (SD:8-21, b = log ℓ², so
    b = 2 log l for CP.R's direct l; a = log k² = 0), chol_solve (KF:25-29), crps (KF:60-68),
    logs (KF:52-57).  R itself is absent, so the R side is unpinned; this pins the algebra."""
    X, Y = T(x).view(len(x), -1), T(y).view(-1, 1)
    n = Y.shape[0]
    out = np.empty((4, len(sd_grid), len(ell_grid)))
    with torch.no_grad():
        for i, sd in enumerate(sd_grid):
            for j, ell in enumerate(ell_grid):
                k_ff = ns["rbf"](X, X, T([0.0]), T([2.0 * math.log(ell)]))
                big_k = k_ff + torch.eye(n) * sd ** 2                              # CP.R:45
                kii = torch.diag(ns["chol_solve"](torch.eye(n), big_k)).view(n, 1)  # CP.R:46
                mean_term = Y - ns["chol_solve"](Y, big_k) / kii                    # CP.R:48
                cov_term = 1 / kii                                                  # CP.R:49
                out[0, i, j] = ns["crps"](mean_term, cov_term, Y).item()           # CP.R:51
                w_mean = k_ff.mm(ns["chol_solve"](Y, big_k))                        # CP.R:58
                w_cov = torch.diag(torch.eye(n) * sd ** 2 + k_ff
                                   - k_ff.mm(ns["chol_solve"](k_ff, big_k))).view(n, 1)  # CP.R:59
                out[1, i, j] = ns["crps"](w_mean, w_cov, Y).item()                 # CP.R:62
                hl = torch.linalg.cholesky(big_k, upper=True).diag().log().sum()  # log(det)/2
                out[2, i, j] = (0.5 * Y.t().mm(ns["chol_solve"](Y, big_k)) + hl
                                + n / 2 * math.log(2 * math.pi)).item()             # CP.R:71
                out[3, i, j] = ns["logs"](mean_term, cov_term + sd ** 2, Y).item()  # CP.R:81-83
    return out


def synth(seed, n, nt, d):
    """SURVEY.md §8(d) synthetic generator."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d))
    Xt = rng.standard_normal((nt, d))
    w = rng.standard_normal(d) / np.sqrt(d)
    y = np.sin(3 * X @ w) + 0.1 * rng.standard_normal(n)
    yt = np.sin(3 * Xt @ w) + 0.1 * rng.standard_normal(nt)
    return X, y, Xt, yt, rng


def simple_data(ns, seed):
    """SIMPLE-DATA generator (SD:158-181) at fp64: x = 2 N(0,1), y ~ MVN(0, rbf + 0.09 I)."""
    torch.manual_seed(seed)
    num_train, num_test, num_va = 120, 300, 30
    num_total = num_train + num_test + num_va
    full_x = 2 * torch.randn(num_total)
    true_log_l_sq = torch.tensor([1.0]).log()
    true_log_k_sq = torch.tensor([1.0]).log()
    k_init = ns["rbf"](full_x.view(num_total, 1), full_x.view(num_total, 1),
                       true_log_k_sq, true_log_l_sq) + torch.eye(num_total) * (0.3 ** 2)
    full_y = torch.distributions.MultivariateNormal(torch.zeros(num_total), k_init).sample()
    X = full_x[:num_train].view(-1, 1).numpy()
    y = full_y[:num_train].numpy()
    Xt = full_x[num_train:num_train + num_test].view(-1, 1).numpy()
    yt = full_y[num_train:num_train + num_test].numpy()
    return X, y, Xt, yt, k_init[:16, :16].numpy()


def main(only=None):
    """only: name prefixes to (re)write (all when None); e.g. `make_goldens.py blockes_ es_`."""
    torch.set_default_dtype(torch.float64)
    ns = load_reference_defs()
    written = []

    def save(name, **arrs):
        if only and not any(name.startswith(p) for p in only):
            return
        path = os.path.join(OUT, name + ".npz")
        np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
        written.append((name, os.path.getsize(path)))

    # ---- L1 building blocks: ARD / rbf Gram samples, chol_solve -------------------
    rng = np.random.default_rng(11)
    Xa, Xb = rng.standard_normal((48, 8)), rng.standard_normal((40, 8))
    ell = np.log(np.linspace(0.6, 2.4, 8))
    ard_ab = ns["ARD"](T(Xa), T(Xb), T([0.3]), T(ell)).numpy()
    ard_aa = ns["ARD"](T(Xa), T(Xa), T([0.3]), T(ell)).numpy()
    ard_iso = ns["ARD"](T(Xa), T(Xb), T([-0.2]), T([0.4])).numpy()
    x1, x2 = rng.standard_normal((30, 1)), rng.standard_normal((25, 1))
    rbf_12 = ns["rbf"](T(x1), T(x2), T([0.1]), T([0.7])).numpy()
    A = ard_aa + 0.05 * np.eye(48)
    Bm = rng.standard_normal((48, 3))
    cs = ns["chol_solve"](T(Bm), T(A)).numpy()
    cs_eye = ns["chol_solve"](torch.eye(48), T(A)).numpy()
    hl = torch.linalg.cholesky(T(A), upper=True).diag().log().sum().item()
    nys_Z = rng.standard_normal((7, 8))
    ns["para_k"], ns["para_l"], ns["dtype"] = T([0.3]), T(ell).view(1, -1), torch.DoubleTensor
    q_ab = ns["Q"](T(Xa), T(nys_Z), T(Xb)).numpy()
    save("l1_blocks", Xa=Xa, Xb=Xb, log_ell=ell, log_sf2=0.3, ard_ab=ard_ab, ard_aa=ard_aa,
         ard_iso=ard_iso, iso_log_sf2=-0.2, iso_log_ell=0.4,
         x1=x1, x2=x2, rbf_12=rbf_12, rbf_log_sf2=0.1, rbf_log_ell2=0.7,
         A=A, B=Bm, chol_solve=cs, chol_solve_eye=cs_eye, half_logdet=hl,
         nys_Z=nys_Z, Q_ab=q_ab)

    # ---- scoring rules on fixed vectors ----------------------------------------
    m = rng.standard_normal(50)
    c = np.exp(rng.standard_normal(50) * 0.5)
    yv = rng.standard_normal(50)
    ytr = rng.standard_normal(70)
    with torch.no_grad():
        sc = {
            "crps": ns["crps"](T(m).view(-1, 1), T(c).view(-1, 1), T(yv).view(-1, 1)).item(),
            "logs": ns["logs"](T(m).view(-1, 1), T(c).view(-1, 1), T(yv).view(-1, 1)).item(),
            "msll": ns["trivial_loss"](T(m).view(-1, 1), T(c).view(-1, 1), T(yv).view(-1, 1),
                                       T(ytr).view(-1, 1)).item(),
            "smse": ns["SMSE"](T(m).view(-1, 1), T(yv).view(-1, 1), T(ytr).view(-1, 1)).item(),
        }
    save("scores", m=m, c=c, y=yv, y_train=ytr, **sc)

    # ---- SIMPLE-DATA style 1-D cases (full GP, ARD at d=1 and rbf) --------------
    for j in (0, 1):
        X, y, Xt, yt, kblk = simple_data(ns, 100 * j)
        for tag, th in (("init", (1.0, 1.0, 1.0)), ("fit", (0.0, 0.0, math.log(0.09)))):
            o = full_case(ns, X, y, Xt, yt, *th, kern="ARD")
            g = grads_full(ns, X, y, *th, kern="ARD")  # SD:199-216: scalar para_l, d = 1
            save(f"sd_j{j}_{tag}", X=X, y=y, Xt=Xt, yt=yt, theta=np.array(th), kern="ARD", **o, **g)
        o = full_case(ns, X, y, Xt, yt, 0.0, 0.5, math.log(0.09), kern="rbf")
        g = grads_full(ns, X, y, 0.0, 0.5, math.log(0.09), kern="rbf")
        save(f"sd_j{j}_rbf", X=X, y=y, Xt=Xt, yt=yt, theta=np.array((0.0, 0.5, math.log(0.09))),
             kern="rbf", k_init_block=kblk, **o, **g)

    # ---- d = 8 synthetic full-GP cases ------------------------------------------
    d = 8
    log_ell8 = np.log(2.0) + 0.15 * (np.arange(d) - 3.5) / 3.5
    for n, nt in ((64, 64), (500, 500), (2000, 500)):
        X, y, Xt, yt, _ = synth(1000 + n, n, nt, d)
        th = (0.0, log_ell8, math.log(0.01))
        o = full_case(ns, X, y, Xt, yt, *th)
        extra = grads_full(ns, X, y, *th) if n <= 500 else {}
        save(f"full_n{n}_d8", X=X, y=y, Xt=Xt, yt=yt, log_sf2=th[0], log_ell=th[1],
             log_sn2=th[2], **o, **extra)

    # ---- scalar length-scale broadcast over d = 8 (KF:8-12 with para_l of shape [1]) ----
    X, y, Xt, yt, _ = synth(1064, 64, 64, d)
    th = (0.2, math.log(1.7), math.log(0.02))
    o = full_case(ns, X, y, Xt, yt, *th)
    save("full_n64_d8_iso", X=X, y=y, Xt=Xt, yt=yt, log_sf2=th[0], log_ell=np.array([th[1]]),
         log_sn2=th[2], **o, **grads_full(ns, X, y, *th))

    # ---- FITC cases -------------------------------------------------------------
    for n, nt, mm, zkind in ((64, 64, 5, "rows"), (500, 500, 20, "rows"),
                             (500, 200, 20, "uniform"), (2000, 500, 200, "rows")):
        X, y, Xt, yt, rng2 = synth(2000 + n + mm, n, nt, d)
        if zkind == "rows":
            Z = X[rng2.choice(n, mm, replace=False)]
        else:  # K20:216 style: inducing_x = torch.rand(m, d)
            Z = rng2.random((mm, d))
        th = (0.0, log_ell8, math.log(0.01))
        o = fitc_case(ns, X, y, Xt, yt, Z, *th)
        extra = grads_fitc(ns, X, y, Z, *th) if n <= 500 else {}
        save(f"fitc_n{n}_m{mm}_{zkind}", X=X, y=y, Xt=Xt, yt=yt, Z=Z, log_sf2=th[0],
             log_ell=th[1], log_sn2=th[2], **o, **extra)

    # ---- FITC with a scalar length-scale (SF-style para_l of shape [1]) and d = 1 -----
    for n, mm, dd, th in ((64, 5, 8, (0.3, math.log(1.5), math.log(0.05))),
                          (120, 5, 1, (0.1, math.log(0.8), math.log(0.09)))):
        X, y, Xt, yt, rng2 = synth(3000 + n + dd, n, 40, dd)
        Z = rng2.random((mm, dd))
        o = fitc_case(ns, X, y, Xt, yt, Z, *th)
        save(f"fitc_n{n}_m{mm}_d{dd}_iso", X=X, y=y, Xt=Xt, yt=yt, Z=Z, log_sf2=th[0],
             log_ell=np.array([th[1]]), log_sn2=th[2], **o,
             **grads_fitc(ns, X, y, Z, *th))

    # ---- next-2: 4-fold block-LOO DSS / KC (equal folds: the scripts' chol_solve(eye(index1),
    # k_f) needs n % 4 == 0) ----------------------------------------------------------
    for n, mm in ((64, 6), (500, 20)):
        X, y, Xt, yt, rng2 = synth(4000 + n, n, 16, d)
        th = (0.1, log_ell8, math.log(0.02))
        Z = X[rng2.choice(n, mm, replace=False)]
        save(f"block_full_n{n}", X=X, y=y, log_sf2=th[0], log_ell=th[1], log_sn2=th[2],
             **block_loo_case(ns, X, y, *th))
        save(f"block_fitc_n{n}_m{mm}", X=X, y=y, Z=Z, log_sf2=th[0], log_ell=th[1],
             log_sn2=th[2], **block_loo_case(ns, X, y, *th, Z=Z))

    # ---- next-2: the energy score (ES KF:70-101) on the 4-fold block-LOO predictive
    # (KF:607-663), the reference's own torch.randn draws replayed -------------------------
    for n, S in ((64, 300), (200, 40)):
        X, y, _, _, _ = synth(5000 + n, n, 16, d)
        th = (0.1, log_ell8, math.log(0.02))
        save(f"blockes_full_n{n}", X=X, y=y, log_sf2=th[0], log_ell=th[1], log_sn2=th[2],
             **es_case(ns, X, y, *th, num_sim=S, seed=7 + n))

    # ---- ES / dss helpers on one fixed Gaussian (compat.ES / compat.dss) -----------------
    rng = np.random.default_rng(23)
    b = 12
    A0 = rng.standard_normal((b, b))
    C = A0 @ A0.T / b + 0.1 * np.eye(b)
    m, yv = rng.standard_normal(b), rng.standard_normal(b)
    with torch.no_grad():
        torch.manual_seed(5)
        es1 = float(ns["ES"](T(m).view(-1, 1), T(C), b, T(yv).view(-1, 1), 40))
        torch.manual_seed(5)
        dr = np.concatenate([torch.randn(40, b).numpy().ravel() for _ in range(2)])
        dss1 = float(ns["dss"](T(m).view(-1, 1), T(C), b, T(yv).view(-1, 1)))
    save("es_single", m=m, C=C, y=yv, num_sim=40, draws=dr, es=es1, dss=dss1)

    # ---- K20's own dss (K20:106-111: cov_term.inverse()) beside KF's (KF:103-108: chol_solve) on
    #      the same Gaussians — a moderately and a badly conditioned covariance (own rng: the
    #      goldens above are untouched)
    rng3 = np.random.default_rng(31)
    cases = {}
    for tag, b, jit in (("well", 24, 0.5), ("ill", 40, 1e-6)):
        Mx = rng3.standard_normal((b, b))
        C = Mx @ Mx.T / b + jit * np.eye(b)
        m, yv = rng3.standard_normal(b), rng3.standard_normal(b)
        with torch.no_grad():
            kf = float(ns["dss"](T(m).view(-1, 1), T(C), b, T(yv).view(-1, 1)))
            k20 = float(ns["dss_k20"](T(m).view(-1, 1), T(C), b, T(yv).view(-1, 1)))
        cases.update({f"{tag}_m": m, f"{tag}_C": C, f"{tag}_y": yv, f"{tag}_dss_kf": kf,
                      f"{tag}_dss_k20": k20})
    save("dss_k20", **cases)

    # ---- contour-plot.R surfaces: n = 20 on CP.R's 50 × 50 grid; a d = 2, n = 100 grid ----
    sys.path.insert(0, os.path.join(os.path.dirname(OUT), "..", "oracle"))
    import gp_oracle as O  # the CP.R data generator only (x = seq(-6, 6, 20), y ~ MVN + noise)
    x, yv = O.cp_data(seed=0)
    l_range, sd_range = np.linspace(0.01, 2.0, 50), np.linspace(0.01, 1.0, 50)
    save("surface_cp", x=x, y=yv, ell=l_range, sd=sd_range,
         surf=surface_case(ns, x, yv, l_range, sd_range))
    rng2 = np.random.default_rng(21)
    x2 = rng2.uniform(-3, 3, (100, 2))
    y2 = np.sin(x2[:, 0]) * np.cos(x2[:, 1]) + 0.1 * rng2.standard_normal(100)
    l2, sd2 = np.array([0.3, 0.7, 1.1, 1.6, 2.4]), np.array([0.05, 0.2, 0.6])
    save("surface_d2", x=x2, y=y2, ell=l2, sd=sd2, surf=surface_case(ns, x2, y2, l2, sd2))

    tot = 0
    for name, sz in written:
        print(f"{name:28s} {sz/1024:8.1f} KiB")
        tot += sz
    print(f"total {tot/1024:.1f} KiB")


if __name__ == "__main__":
    main(sys.argv[1:] or None)
