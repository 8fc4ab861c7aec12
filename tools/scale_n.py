"""Full-GP unit (fit + predict + score, C3's shape ratios: d = 8, n* = n/4) at growing n on one
MI355X: wall ms per unit and the unit's algorithmic rate 2n³/3 + n²n* over it — how the
latency-bound bottom of the recursion amortises as n grows, with the n² buffers (A, L⁻¹,
workspace, K*f: ~21 n² bytes) held in HBM.  (n_pad² stays below 2³¹ elements up to n = 46 080.)   python tools/scale_n.py [n ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))

import bench  # noqa: E402
import gpscore  # noqa: E402

ns = [int(a) for a in sys.argv[1:]] or [10000, 20000, 30000, 40000, 46000]
ctx = gpscore.Context(0)
print("%7s %7s %10s %10s %9s %8s" % ("n", "n*", "ms/unit", "TF/s alg", "of peak", "HBM GB"), flush=True)
for n in ns:
    nt = n // 4
    X, y, Xt, yt, _, th = bench.synth(n, 8, nt, 3)
    gp = gpscore.GP(ctx=ctx)
    gp.set_data(X, y)
    gp.set_test(Xt, yt)

    def unit():
        gp.fit(theta=th, return_loo=False)
        return gp.predict(with_scores=True)
    unit()
    reps = 3 if n <= 40000 else 2
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        unit()
    ctx.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / reps
    flop = 2.0 * n ** 3 / 3.0 + float(n) ** 2 * nt
    npad = -(-n // 128) * 128
    gb = (2 * npad * npad + npad * npad / 3 + (nt + 127) // 128 * 128 * npad) * 8 / 1e9
    print("%7d %7d %10.1f %10.2f %8.1f%% %8.1f" % (n, nt, ms, flop / ms / 1e9, 100 * flop / ms / 1e9 / 78.6, gb),
          flush=True)
    del gp
