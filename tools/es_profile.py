"""Per-kernel breakdown of one C2 energy-score GD iteration (value + gradient, 4 folds of 1250,
300 draws per fold; KF:607-663) from the library's hipEvent records (one stream)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))
import bench  # noqa: E402
import gpscore  # noqa: E402
from gpscore.gp import es_draws  # noqa: E402

c = bench.CONFIGS["C2"]
X, y, _, _, _, th = bench.synth(c["n"], c["d"], c["nt"], c["seed"])
ctx = gpscore.Context(0)
gp = gpscore.GP(ctx=ctx)
gp.set_data(X, y)
draws = es_draws(c["n"], 4, 300, np.random.default_rng(0))
for obj in sys.argv[1:] or ["es"]:
    kw = {"num_sim": 300, "draws": draws} if obj == "es" else {}
    gp.block_loo(th, obj, grad=True, **kw)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        gp.block_loo(th, obj, grad=True, **kw)
    ctx.synchronize()
    print(f"{obj}: {1e3 * (time.perf_counter() - t0) / 3:.2f} ms per iteration (production)")
    if os.environ.get("ES_PROF_SINGLE"):
        ctx.set_overlap(False)
    ctx.prof(2)
    gp.block_loo(th, obj, grad=True, **kw)
    rep = ctx.prof_collect()
    ctx.prof(False)
    ctx.set_overlap(True)
    tot = sum(v["ms"] for v in rep.values())
    print(f"  kernels (summed launch times): {tot:.2f} ms")
    for k, v in sorted(rep.items(), key=lambda kv: -kv[1]["ms"])[:25]:
        tf = v["flop"] / (v["ms"] * 1e-3) / 1e12 if v["flop"] and v["ms"] else 0.0
        print(f"  {k:60s} n={v['count']:4d} {v['ms']:8.3f} ms {tf:6.1f} TF")
