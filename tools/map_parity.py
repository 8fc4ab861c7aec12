"""Tile orders are scheduling only: a unit under GPS_OPT_GEMM_MAP=<m> must reproduce the
default order's outputs bitwise (same tiles, same K loops).  python tools/map_parity.py 5"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import gpscore  # noqa: E402
from gpscore import _lib  # noqa: E402

mode = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ctx = gpscore.Context(0)
bad = 0
for name, (n, nt, m) in {"full": (6016, 1500, None), "fitc": (20000, 3000, 1500)}.items():
    X, y, Xt, yt, Z, th = bench.synth(n, 8, nt, 7, m)
    outs = []
    for mm in (0, mode):
        ctx.call("gps_ctx_set_option", _lib.GPS_OPT_GEMM_MAP, mm)
        gp = gpscore.GP(ctx=ctx)
        gp.set_data(X, y, kind=name, Z=Z)
        gp.set_test(Xt, yt)
        r = gp.fit(theta=th)
        mu, var = gp.predict()
        outs.append((r.mu_loo, r.var_loo, mu, var, r.objectives["nlml"]))
    same = all(np.array_equal(a, b) for a, b in zip(outs[0][:4], outs[1][:4])) and outs[0][4] == outs[1][4]
    print(name, "map", mode, "bitwise equal to map 0:", same, flush=True)
    bad += not same
ctx.call("gps_ctx_set_option", _lib.GPS_OPT_GEMM_MAP, 0)
sys.exit(1 if bad else 0)
