"""Small-n full-GP fits with the persistent factorisation on / off (diagnostics)."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT + "/scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd")
import gpscore
ctx = gpscore.Context(0)
rng = np.random.default_rng(8)
for n, d in ((300, 4), (384, 4), (300, 8), (500, 4), (257, 4), (640, 4), (260, 2)):
    X = rng.standard_normal((n, d)); y = np.sin(X.sum(1))
    th = (0.0, 0.0, np.log(0.05))
    out = []
    for dag, graph in ((0, 1), (1, 1), (1, 0)):
        ctx.set_dag(bool(dag), 20); ctx.call("gps_ctx_set_option", 10, graph)
        gp = gpscore.GP(ctx=ctx)
        r = gp.fit(X, y, th)
        out.append((r.objectives["nlml"], r.objectives["loo_crps"], int(np.isnan(r.mu_loo).sum()),
                    int(np.isnan(r.var_loo).sum()), int(np.nanargmax(np.isnan(r.var_loo))) if np.isnan(r.var_loo).any() else -1))
    print(n, d, out, flush=True)
