"""Which GPU intermediate carries the FITC block-LOO gradient's extra rounding noise (VERDICT r5
next 4)?  The case is test_gpu_shards.test_fitc_blockloo_shards[4-4-kc]'s (n = 4000,
m = 40, d = 4, KC over 4 folds, θ- and Z-gradient; K20:655-720).

1. Floors: the gradient's change under 1e-15 relative input perturbations, GPU and CPU oracle.
2. The GPU's intermediates (gps_fitc_intermediates: K̃mm, Lm⁻¹, Knm, λ, Lb⁻¹) against the
   oracle's (numpy / LAPACK fp64), normwise.
3. Each GPU intermediate fed alone into the oracle's whitened gradient (the rest of the oracle
   unchanged; λ is recomputed from a substituted Knm / Lm⁻¹ unless λ itself is substituted): how
   far the gradient moves from the oracle's own.  The intermediate whose substitution moves it by
   the GPU's excess over the oracle floor is the one to fix.
Prints a JSON record.  Usage (GPU): python tools/fitc_noise_localise.py [out.json [intermediates.npz]]
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd")]

import gp_oracle as O  # noqa: E402
import gpscore  # noqa: E402
from gpscore import _lib  # noqa: E402
from test_gpu_shards import _case  # noqa: E402


def nrel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / np.max(np.abs(np.asarray(b))))


X, y, _, _, Z, th = _case(4000, 10, 40, 4, 49)
n, m = len(y), len(Z)
gp = gpscore.GP()


def gpu(Xp, Zp):
    gp.set_data(Xp, y, kind="fitc", Z=Zp)
    v, g, _, gz = gp.block_loo(th, "kc", nfold=4, grad=True)
    return float(v), np.asarray(g, float), np.asarray(gz, float)


def oracle(Xp, Zp):
    v, g, gz = O.fast_fitc_blockloo(Xp, y, Zp, *th, "kc", nfold=4, want_grad=True)
    return float(v), np.asarray(g, float), np.asarray(gz, float)


rec = {"case": "test_fitc_blockloo_shards[4-4-kc] inputs, unsharded: n=4000 m=40 d=4 KC, 4 folds"}
g0 = gpu(X, Z)
KnmG, lamG = np.zeros((n, m)), np.zeros(n)
LmG, LbG, KmmG = np.zeros((m, m)), np.zeros((m, m)), np.zeros((m, m))
P = _lib.ptr
gp.ctx.call("gps_fitc_intermediates", P(KnmG), P(lamG), P(LmG), P(LbG), P(KmmG))
o0 = oracle(X, Z)
rec["gpu_vs_oracle"] = {"grad": nrel(g0[1], o0[1]), "grad_Z": nrel(g0[2], o0[2])}
for name, fn in (("gpu_floor", gpu), ("oracle_floor", oracle)):
    base = g0 if fn is gpu else o0
    fl = []
    for seed in (1, 2):
        rng = np.random.default_rng(seed)
        r = fn(X * (1 + 1e-15 * rng.standard_normal(X.shape)), Z * (1 + 1e-15 * rng.standard_normal(Z.shape)))
        fl.append({"grad": nrel(r[1], base[1]), "grad_Z": nrel(r[2], base[2])})
    rec[name] = fl

# the oracle's own intermediates
KmmO, LmO, _ = O.fitc_shared(Z, th[0], th[1])
partO = O.fitc_partials(X, y, Z, LmO, *th)
LbO, _, _ = O.fitc_finish_shared(KmmO, partO["B"], partO["b"])
rec["intermediate_diff"] = {"Kmm": nrel(KmmG, KmmO), "Lm_inv": nrel(np.tril(LmG), LmO),
                            "Knm": nrel(KnmG, partO["_Knm"]), "lam": nrel(lamG, partO["_lam"]),
                            "Lb_inv": nrel(np.tril(LbG), LbO)}
# λ_i = sf² − q_i + σ² cancels to ~σ² near an inducing point: its relative error in ulps there
rec["lam_rel_max"] = float(np.max(np.abs(lamG - partO["_lam"]) / partO["_lam"]))

orig = {k: getattr(O, k) for k in ("fitc_shared", "fitc_partials", "fitc_finish_shared")}


def with_gpu(names):
    def shared(Zp, a, b):
        K, L, ld = orig["fitc_shared"](Zp, a, b)
        if "Kmm" in names:
            K = KmmG.copy()
            _, L, ld = O.fast_potrf_inv(K)
        if "Lm_inv" in names:
            L = np.tril(LmG)
        return K, L, ld

    def partials(Xp, yy, Zp, Lm_inv, a, b, c):
        p = orig["fitc_partials"](Xp, yy, Zp, Lm_inv, a, b, c)
        K = KnmG.copy() if "Knm" in names else p["_Knm"]
        if "lam" in names:
            lam = lamG.copy()
        else:
            W = K @ Lm_inv.T
            lam = math.exp(a) - np.sum(W * W, axis=1) + math.exp(c)
        yy = np.asarray(yy, float).ravel()
        Ks = K / lam[:, None]
        return {"B": K.T @ Ks, "b": Ks.T @ yy, "s": np.array([np.sum(np.log(lam)), np.sum(yy * yy / lam)]),
                "_Knm": K, "_lam": lam}

    def finish(Kmm, B, b):
        Lb, ld, c = orig["fitc_finish_shared"](Kmm, B, b)
        if "Lb_inv" in names:
            Lb = np.tril(LbG)
            c = Lb.T @ (Lb @ b)
        return Lb, ld, c

    O.fitc_shared, O.fitc_partials, O.fitc_finish_shared = shared, partials, finish
    try:
        return oracle(X, Z)
    finally:
        for k, v in orig.items():
            setattr(O, k, v)


sub = {}
for names in (("Kmm",), ("Lm_inv",), ("Knm",), ("lam",), ("Lb_inv",), ("Kmm", "Knm"),
              ("Kmm", "Lm_inv", "Knm", "lam", "Lb_inv")):
    r = with_gpu(names)
    sub["+".join(names)] = {"grad_vs_oracle": nrel(r[1], o0[1]), "gradZ_vs_oracle": nrel(r[2], o0[2]),
                            "grad_vs_gpu": nrel(r[1], g0[1])}
rec["substituted"] = sub

# 4. the floor itself: at 1e-15-perturbed inputs, how far each GPU intermediate moves from its value
#    at the base inputs (GPU) against the oracle's own intermediate's move, and whether the oracle
#    fed the GPU's perturbed Lb⁻¹ alone reproduces the GPU's perturbed gradient
save = {"Knm": KnmG, "lam": lamG, "Lm_inv": LmG, "Lb_inv": LbG, "Kmm": KmmG}
moves = []
for seed in (1, 2):
    rng = np.random.default_rng(seed)
    Xp = X * (1 + 1e-15 * rng.standard_normal(X.shape))
    Zp = Z * (1 + 1e-15 * rng.standard_normal(Z.shape))
    gp_ = gpu(Xp, Zp)
    K2, l2, Lm2, Lb2, Km2 = (np.zeros_like(a) for a in (KnmG, lamG, LmG, LbG, KmmG))
    gp.ctx.call("gps_fitc_intermediates", P(K2), P(l2), P(Lm2), P(Lb2), P(Km2))
    KmmO2, LmO2, _ = O.fitc_shared(Zp, th[0], th[1])
    partO2 = O.fitc_partials(Xp, y, Zp, LmO2, *th)
    LbO2, _, _ = O.fitc_finish_shared(KmmO2, partO2["B"], partO2["b"])
    mv = {"gpu": {"Lm_inv": nrel(np.tril(Lm2), np.tril(LmG)), "lam": nrel(l2, lamG),
                  "Lb_inv": nrel(np.tril(Lb2), np.tril(LbG)), "Knm": nrel(K2, KnmG)},
          "oracle": {"Lm_inv": nrel(LmO2, LmO), "lam": nrel(partO2["_lam"], partO["_lam"]),
                     "Lb_inv": nrel(LbO2, LbO), "Knm": nrel(partO2["_Knm"], partO["_Knm"])}}
    KnmG_b, lamG_b, LmG_b, LbG_b, KmmG_b = KnmG, lamG, LmG, LbG, KmmG
    KnmG, lamG, LmG, LbG, KmmG = K2, l2, Lm2, Lb2, Km2
    X_b, Z_b = X, Z
    X, Z = Xp, Zp
    r = with_gpu(("Lb_inv",))
    r_all = with_gpu(("Kmm", "Lm_inv", "Knm", "lam", "Lb_inv"))
    X, Z = X_b, Z_b
    KnmG, lamG, LmG, LbG, KmmG = KnmG_b, lamG_b, LmG_b, LbG_b, KmmG_b
    mv["gpu_perturbed_grad_vs_oracle_with_its_Lb_inv"] = nrel(r[1], gp_[1])
    mv["gpu_perturbed_grad_vs_oracle_with_all"] = nrel(r_all[1], gp_[1])
    moves.append(mv)
    save[f"Lb_inv_p{seed}"] = Lb2
rec["perturbation_moves"] = moves
if len(sys.argv) > 2:
    np.savez_compressed(sys.argv[2], **save)
out = json.dumps(rec, indent=1)
print(out)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(out)
