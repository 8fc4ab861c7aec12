"""Run the C3 (or --config) production unit a few times with library options set, for a
rocprofv3 --kernel-trace of the schedule (tools/critpath.py reads the trace).
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o run -- \\
      python3 tools/trace_unit.py side=4 persist=448"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))

import bench  # noqa: E402
import gpscore  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_bench import KEYS  # noqa: E402

cfg = "C3"
opts = []
for a in sys.argv[1:]:
    k, v = a.split("=")
    if k == "config":
        cfg = v
    else:
        opts.append((KEYS[k], int(v)))
c = bench.CONFIGS[cfg]
ctx = gpscore.Context(0)
for k, v in opts:
    ctx.call("gps_ctx_set_option", k, v)
gp = gpscore.GP(ctx=ctx)
X, y, Xt, yt, Z, th = bench.synth(c["n"], c["d"], c["nt"], c["seed"], c.get("m"))
if Z is None:
    gp.set_data(X, y)
else:
    gp.set_data(X, y, kind="fitc", Z=Z)
gp.set_test(Xt, yt)
for _ in range(3):
    gp.fit(theta=th, return_loo=False)
    gp.predict(with_scores=True)
ctx.synchronize()
print("done")
