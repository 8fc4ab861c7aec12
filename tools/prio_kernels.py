# prof-mode kernel classes at C3 per GPS_OPT_GEMM_PRIO setting (single stream, eager)
import os, sys
ROOT = os.getcwd()
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))
import bench, gpscore
from gpscore import _lib
c = bench.CONFIGS["C3"]
X, y, Xt, yt, Z, th = bench.synth(c["n"], c["d"], c["nt"], c["seed"], None)
ctx = gpscore.Context(0)
gp = gpscore.GP(ctx=ctx)
gp.set_data(X, y); gp.set_test(Xt, yt)
gp.fit(theta=th, return_loo=False)
for rnd in range(2):
    for pr in (0, 1, 3):
        ctx.call("gps_ctx_set_option", _lib.GPS_OPT_GEMM_PRIO, pr)
        ctx.prof(True)
        gp.fit(theta=th, return_loo=False); gp.predict()
        rep = ctx.prof_collect(); ctx.prof(False)
        print(rnd, "prio", pr, " ".join("%s %.2f" % (k, rep[k]["ms"]) for k in ("gemm_trmm_l", "gemm_syrk_l", "gemm_trmm_colred") if k in rep), flush=True)
