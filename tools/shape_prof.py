"""Per-shape GEMM accounting of one bench unit (gps_prof_enable level 2: every launch tagged
with its layouts, M×N×K, triangular form, tile and split), overlap off, sorted by time.

  python tools/shape_prof.py --config C3
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))

import bench  # noqa: E402
import gpscore  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    c = bench.CONFIGS[args.config]
    ctx = gpscore.Context(0)
    gp = gpscore.GP(ctx=ctx)
    X, y, Xt, yt, Z, th = bench.synth(c["n"], c["d"], c["nt"], c["seed"], c.get("m"))
    if Z is None:
        gp.set_data(X, y)
    else:
        gp.set_data(X, y, kind="fitc", Z=Z)
    gp.set_test(Xt, yt)

    def unit():
        gp.fit(theta=th, return_loo=False)
        gp.predict(with_scores=True)
    unit()
    ctx.set_overlap(False)
    ctx.call("gps_prof_enable", 2)
    for _ in range(args.steps):
        unit()
    ctx.synchronize()
    prof = ctx.prof_collect()
    ctx.call("gps_prof_enable", 0)
    tot = sum(v["ms"] for v in prof.values()) / args.steps
    print("total %.2f ms per unit over %d tags" % (tot, len(prof)))
    for tag, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"]):
        ms = v["ms"] / args.steps
        tf = v["flop"] / (v["ms"] * 1e-3) / 1e12 if v["flop"] and v["ms"] else 0.0
        print("%-70s n=%5.1f %9.3f ms %6.1f TF/s" % (tag, v["count"] / args.steps, ms, tf))


if __name__ == "__main__":
    main()
