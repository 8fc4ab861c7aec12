"""Per-launch-shape accounting of one bench unit (tools/shape_prof.py [--config C3] [--fitc]).

Runs the bench workload with overlap off and gps_prof_enable(ctx, 2), so every GEMM
tag carries layout / MxNxK / triangular mode / split-K / lda, and prints the shapes
sorted by time with their achieved TF/s.  Diagnostic only (not part of the bench).
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
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--grad", default=None, help="profile value_and_grad(objective) instead")
    ap.add_argument("--block", default=None,
                    help="profile block_loo(objective, grad=True) (dss / kc / es; ES: 300 draws)")
    args = ap.parse_args()
    c = bench.CONFIGS[args.config]
    ctx = gpscore.Context(0)
    gp = gpscore.GP(ctx=ctx)
    X, y, Xt, yt, Z, th = bench.synth(c["n"], c["d"], c["nt"], c["seed"], c.get("m"))
    if Z is None:
        gp.set_data(X, y)
        gp.set_test(Xt, yt)

        def unit():
            gp.fit(theta=th, return_loo=False)
            gp.predict(with_scores=True)
    else:
        gp.set_data(X, y, kind="fitc", Z=Z)
        gp.set_test(Xt, yt)

        def unit():
            gp.fit(theta=th, return_loo=False)
            gp.predict(with_scores=True)
    if args.grad:
        def unit():  # noqa: F811
            gp.value_and_grad(th, args.grad)
    if args.block:
        kw = {}
        if args.block == "es":
            import numpy as np
            from gpscore.gp import es_draws
            kw = {"num_sim": 300, "draws": es_draws(c["n"], 4, 300, np.random.default_rng(0))}

        def unit():  # noqa: F811
            gp.block_loo(th, args.block, grad=True, **kw)
    unit()
    ctx.synchronize()
    ctx.set_overlap(False)
    ctx.call("gps_prof_enable", 2)
    for _ in range(args.steps):
        unit()
    prof = ctx.prof_collect()
    tot = sum(v["ms"] for v in prof.values()) / args.steps
    print("total kernel ms/unit %.3f" % tot)
    rows = sorted(prof.items(), key=lambda kv: -kv[1]["ms"])
    for tag, v in rows[: args.top]:
        ms = v["ms"] / args.steps
        tf = v["flop"] / (v["ms"] * 1e-3) / 1e12 if v["flop"] and v["ms"] else 0.0
        print("%-58s n=%5.1f %9.3f ms  avg %8.1f us  %5.1f TF" % (
            tag, v["count"] / args.steps, ms, 1e3 * ms / (v["count"] / args.steps), tf))


if __name__ == "__main__":
    main()
