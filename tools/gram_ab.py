"""Gram kernel timings (gram_kff / gram_ksf at C3, gram_knm at C5) of the library this process
loads (GPSCORE_LIB selects a variant build): hipEvent records over 5 fits, single stream, for
each GPS_OPT_GRAM_REG mode given on the command line (default: 1 2)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))
import bench  # noqa: E402
import gpscore  # noqa: E402

ctx = gpscore.Context(0)
out = {"lib": os.environ.get("GPSCORE_LIB", "in-tree")}
modes = [int(a) for a in sys.argv[1:]] or [1, 2]
for cfg, mode in [(c, md) for c in ("C3", "C5") for md in modes]:
    ctx.set_gram_reg(mode)
    c = bench.CONFIGS[cfg]
    X, y, Xt, yt, Z, th = bench.synth(c["n"], c["d"], c["nt"], c["seed"], c.get("m"))
    gp = gpscore.GP(ctx=ctx)
    if Z is None:
        gp.set_data(X, y)
    else:
        gp.set_data(X, y, kind="fitc", Z=Z)
    gp.set_test(Xt, yt)
    gp.fit(theta=th, return_loo=False)
    ctx.set_overlap(False)
    ctx.prof(True)
    reps = int(os.environ.get("GRAM_AB_REPS", "5"))
    for _ in range(reps):
        gp.fit(theta=th, return_loo=False)
        gp.predict()
    rep = ctx.prof_collect()
    ctx.prof(False)
    ctx.set_overlap(True)
    for k, v in rep.items():
        if k.startswith("gram"):
            out[f"{cfg}.{k}.mode{mode}"] = {"ms": v["ms"] / v["count"], "GB/s": v["bytes"] / (v["ms"] * 1e-3) / 1e9,
                                            **({"max_ms": v["max_ms"]} if "max_ms" in v else {})}
print(json.dumps(out))
