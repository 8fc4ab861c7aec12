"""One FITC C4 unit (fit + predict + score) on cuda:0 — the program the C4 counter passes of
tools/profile_round.sh profile (every dispatch serialised and sampled, so one warm-up unit
and one measured unit; traffic.py averages per kernel name over both)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))

import bench  # noqa: E402
import gpscore  # noqa: E402

c = bench.CONFIGS["C4"]
X, y, Xt, yt, Z, th = bench.synth(c["n"], c["d"], c["nt"], c["seed"], c["m"])
gp = gpscore.GP()
if os.environ.get("GPS_SLAB_XCD"):  # A/B of GPS_OPT_SLAB_XCD under the counter passes
    from gpscore import _lib
    gp.ctx.call("gps_ctx_set_option", _lib.GPS_OPT_SLAB_XCD, int(os.environ["GPS_SLAB_XCD"]))
gp.set_data(X, y, kind="fitc", Z=Z)
gp.set_test(Xt, yt)
for _ in range(2):
    gp.fit(theta=th, return_loo=False)
    gp.predict(with_scores=True)
gp.ctx.synchronize()
print("fitc C4 units done")
