"""Round 5: where the FITC block-LOO θ-gradient's perturbation floor comes from, on the
CPU oracle.  Part 1: the oracle gradient under 1e-15 relative input perturbations (the GPU test's
floor measurement, test_gpu_shards.test_fitc_blockloo_shards[4-4-kc]).  Part 2: a half-ulp (1e-16)
relative perturbation of ONE intermediate (λ, Knm, B, Lb⁻¹, Lm⁻¹) and the gradient change it causes.
Usage: python tools/fitc_floor_probe.py"""
import sys
import numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import gp_oracle as O
from test_gpu_shards import _case
X, y, _, _, Z, th = _case(4000, 10, 40, 4, 49)
def run(Xp, Zp, obj="kc"):
    v, g, gz = O.fast_fitc_blockloo(Xp, y, Zp, *th, obj, nfold=4, want_grad=True)
    return v, g, gz
v0, g0, gz0 = run(X, Z)
def nrel(a,b): return np.max(np.abs(a-b))/np.max(np.abs(b))
print("grad", g0)
for seed in (1,2,3):
    rng = np.random.default_rng(seed)
    v,g,gz = run(X*(1+1e-15*rng.standard_normal(X.shape)), Z*(1+1e-15*rng.standard_normal(Z.shape)))
    print("seed", seed, "value %.2e grad %.2e gradZ %.2e" % (abs(v-v0)/abs(v0), nrel(g,g0), nrel(gz,gz0)))
# which component moves?
rng = np.random.default_rng(1)
v,g,gz = run(X*(1+1e-15*rng.standard_normal(X.shape)), Z*(1+1e-15*rng.standard_normal(Z.shape)))
print("per-component rel", np.abs(g-g0)/np.abs(g0))

base = O.fast_fitc_blockloo(X, y, Z, *th, "kc", nfold=4, want_grad=True)
import math
orig = {k: getattr(O, k) for k in ("fitc_partials", "fitc_finish_shared", "fitc_shared", "fast_gram")}
def noisy(a, eps, seed):
    r = np.random.default_rng(seed)
    return a * (1 + eps * r.standard_normal(np.shape(a)))
def run_with(target, eps=1e-16, seed=0):
    if target == "lam":
        def fp(*a, **k):
            p = orig["fitc_partials"](*a, **k); lam = noisy(p["_lam"], eps, seed)
            Knm = p["_Knm"]; yy = np.asarray(a[1]).ravel(); Ks = Knm / lam[:, None]
            return {"B": Knm.T @ Ks, "b": Ks.T @ yy, "s": p["s"], "_Knm": Knm, "_lam": lam}
        O.fitc_partials = fp
    elif target == "Lb_inv":
        def ff(Kmm, B, b):
            Lb, ld, c = orig["fitc_finish_shared"](Kmm, B, b); Lb = noisy(Lb, eps, seed)
            return Lb, ld, Lb.T @ (Lb @ b)
        O.fitc_finish_shared = ff
    elif target == "B":
        def ff(Kmm, B, b):
            return orig["fitc_finish_shared"](Kmm, noisy(B, eps, seed) , b)
        O.fitc_finish_shared = ff
    elif target == "Lm_inv":
        def fs(Z, a, b):
            K, L, ld = orig["fitc_shared"](Z, a, b); return K, noisy(L, eps, seed), ld
        O.fitc_shared = fs
    elif target == "Knm":
        def fg(x, xp, *a, **k):
            G = orig["fast_gram"](x, xp, *a, **k)
            return noisy(G, eps, seed) if G.shape[0] != G.shape[1] else G
        O.fast_gram = fg
    try:
        return O.fast_fitc_blockloo(X, y, Z, *th, "kc", nfold=4, want_grad=True)
    finally:
        for k, v in orig.items(): setattr(O, k, v)
for t in ("lam", "Knm", "B", "Lb_inv", "Lm_inv"):
    errs = []
    for sd in (0, 1):
        v, g, gz = run_with(t, 1e-16, sd)
        errs.append((nrel(g, base[1]), nrel(gz, base[2])))
    print("%-7s eps=1e-16: grad %.2e %.2e  gradZ %.2e %.2e" % (t, errs[0][0], errs[1][0], errs[0][1], errs[1][1]))
