"""Repro of the r3 suite failure: a full-GP factorisation graph captured in one call, replayed
after other work, leaving Linv / logdiag unwritten (diagnostics)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT + "/scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd")
sys.path.insert(0, ROOT + "/tests")
import gpscore
from gpscore._lib import ptr

variant = sys.argv[1] if len(sys.argv) > 1 else "base"
ctx = gpscore.Context(0)
if variant == "nodag":
    ctx.set_dag(False)
from conftest import load_golden, theta_of
g = load_golden("full_n2000_d8")
thg, _ = theta_of(g)
gpw = gpscore.GP(ctx=ctx)
gpw.fit(g["X"], g["y"], thg)  # buffers at their largest first (as in the suite)
rng = np.random.default_rng(4)
th8 = np.array([0.0, 0.3, np.log(0.01)])
X8, Xt8, y8 = rng.standard_normal((300, 8)), rng.standard_normal((1000, 8)), rng.standard_normal(300)
X16, y16 = rng.standard_normal((300, 16)), rng.standard_normal(300)
out = np.zeros(8)
ctx.call("gps_full_set_data", ptr(X8), ptr(y8), 300, 8)
ctx.call("gps_full_set_test", ptr(Xt8), None, 1000)
ctx.call("gps_full_set_data", ptr(X16), ptr(y16), 300, 16)
ctx.call("gps_full_fit", 0, ptr(th8), 1, ptr(out), None, None)
print("capture fit:", out[:5], flush=True)
if variant != "noprof":
    gp = gpscore.GP(ctx=ctx)
    ctx.prof(variant != "fit2000")
    gp.fit(g["X"], g["y"], thg)
    gp.predict(g["Xt"], g["yt"])
    if variant != "fit2000":
        ctx.prof_collect()
    ctx.prof(False)
rng = np.random.default_rng(8)
Xa = rng.standard_normal((300, 4)); ya = np.sin(Xa.sum(1))
th = (0.0, 0.0, np.log(0.05))
a = gpscore.GP(ctx=ctx)
a.set_data(Xa, ya)
a.set_test(Xa[:20])
ra = a.fit(theta=th)
print(variant, "replayed fit:", ra.objectives, flush=True)
ctx.call("gps_ctx_set_option", 10, 0)
print(variant, "eager fit:   ", a.fit(theta=th).objectives, flush=True)
