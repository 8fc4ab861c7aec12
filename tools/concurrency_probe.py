"""How much of the predictive TRMM can hide under the factorisation's latency-bound
phases?  Two independent contexts on one GPU (own streams), C3 sizes: time fit alone,
predict alone (repeated so it spans the fit), and both concurrently from two host
threads (ctypes releases the GIL).  Timing experiment only (no data dependency between
the two).  Usage: python tools/concurrency_probe.py"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))
import gpscore  # noqa: E402

rng = np.random.default_rng(3)
n, nt, d = 20000, 5000, 8
X, Xt = rng.standard_normal((n, d)), rng.standard_normal((nt, d))
y = np.sin(X.sum(1) / 3) + 0.1 * rng.standard_normal(n)
th = (0.0, np.log(2.0) * np.ones(d), np.log(0.01))
ca, cb = gpscore.Context(0), gpscore.Context(0)
ga, gb = gpscore.GP(ctx=ca), gpscore.GP(ctx=cb)
ga.set_data(X, y)
gb.set_data(X, y)
gb.set_test(Xt)
gb.fit(theta=th, return_loo=False)


def fit():
    ga.fit(theta=th, return_loo=False)


def pred(k):
    for _ in range(k):
        gb.predict()


def t(f, *a):
    ca.synchronize()
    cb.synchronize()
    t0 = time.perf_counter()
    f(*a)
    ca.synchronize()
    cb.synchronize()
    return 1e3 * (time.perf_counter() - t0)


EXCL = int(sys.argv[1]) if len(sys.argv) > 1 else 0
if EXCL:  # the predict context's stream leaves the top EXCL CU ids to the fit
    cb.call("gps_ctx_set_option", gpscore._lib.GPS_OPT_MAIN_CU_EXCLUDE, EXCL)
print(f"predict stream excludes {EXCL} CUs")
for _ in range(2):
    fit()
    pred(1)
tf = min(t(fit) for _ in range(3))
tp = min(t(pred, 1) for _ in range(3))
print(f"fit alone {tf:.1f} ms   predict alone {tp:.1f} ms   sequential sum {tf + tp:.1f} ms")
for k in (1, 2, 3):
    res = []
    for _ in range(3):
        def both():
            th_ = threading.Thread(target=pred, args=(k,))
            th_.start()
            fit()
            th_.join()
        res.append(t(both))
    print(f"fit || {k} x predict: {min(res):.1f} ms  (sequential {tf + k * tp:.1f}, "
          f"hidden {tf + k * tp - min(res):.1f} ms)")
