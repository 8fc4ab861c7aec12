"""Same-box A/B of library schedule options on a bench workload (MI355X boxes differ by
~5% in GEMM clocks, so variants must be compared inside one run).

  python tools/ab_bench.py --config C3 map=0 map=4 ov=0
  options: map (GPS_OPT_GEMM_MAP), ov (GPS_OPT_OVERLAP),
           graph (GPS_OPT_GRAPH), tiny (GPS_OPT_TINY_GEMM),
           pre (GPS_OPT_PRED_PRE), dag (GPS_OPT_DAG), dagt (GPS_OPT_DAG_TILES), dep (GPS_OPT_FITC_DEP)
Variants are interleaved round-robin for --rounds rounds; prints the median ms/unit.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402
import gpscore  # noqa: E402
from gpscore import _lib  # noqa: E402

KEYS = {"map": _lib.GPS_OPT_GEMM_MAP, "ov": _lib.GPS_OPT_OVERLAP,
        "graph": _lib.GPS_OPT_GRAPH, "tiny": _lib.GPS_OPT_TINY_GEMM, "pre": _lib.GPS_OPT_PRED_PRE,
        "dag": _lib.GPS_OPT_DAG, "dagt": _lib.GPS_OPT_DAG_TILES, "arch": _lib.GPS_OPT_AR_CHUNKS, "dagg": _lib.GPS_OPT_DAG_GROUP, "sk": _lib.GPS_OPT_STREAM_K, "dagwg": _lib.GPS_OPT_DAG_WGS, "order": _lib.GPS_OPT_DAG_ORDER, "sxcd": _lib.GPS_OPT_SLAB_XCD, "dep": _lib.GPS_OPT_FITC_DEP}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--block", default=None,
                    help="time block_loo(objective, grad=True) (dss / kc / es; ES: 300 draws)")
    ap.add_argument("--phases", action="store_true",
                    help="also one pass per variant and round with gps_phase_enable (FITC forward phases)")
    ap.add_argument("variants", nargs="+")
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
    if args.block:
        kw = {}
        if args.block == "es":
            from gpscore.gp import es_draws
            kw = {"num_sim": 300, "draws": es_draws(c["n"], 4, 300, np.random.default_rng(0))}

        def unit():  # noqa: F811
            gp.block_loo(th, args.block, grad=True, **kw)

    variants = []
    for v in args.variants:
        opts = {}
        for kv in v.split(","):
            k, val = kv.split("=")
            opts[KEYS[k]] = int(val)
        variants.append((v, opts))
    unit()
    times = {v: [] for v, _ in variants}
    phs = {v: [] for v, _ in variants}
    defaults = {KEYS["dagwg"]: 0}  # options a variant sets and the next one might not (reset first)
    for _ in range(args.rounds):
        for name, opts in variants:
            for key, val in {**defaults, **opts}.items():
                ctx.call("gps_ctx_set_option", key, val)
            unit()
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                unit()
            ctx.synchronize()
            times[name].append(1e3 * (time.perf_counter() - t0) / args.steps)
            if args.phases:
                ctx.phases(True)
                unit()
                ctx.phases(False)
                phs[name].append({k: v["ms"] for k, v in ctx.phase_collect()["phases"].items()})
    for name, _ in variants:
        ts = times[name]
        print("%-24s median %8.2f ms/unit  (all: %s)" % (name, float(np.median(ts)),
                                                        " ".join("%.2f" % t for t in ts)))
        if phs[name]:
            keys = phs[name][0].keys()
            print("    phases (median ms): " + " ".join("%s %.3f" % (k, float(np.median([p[k] for p in phs[name]])))
                                                   for k in keys))


if __name__ == "__main__":
    main()
