"""Cost of the reference-shaped compat surface (gpscore.compat: host arrays in and out per
call, the scripts' own op sequence) against the device-resident GP path, on one GPU.
One line per (n, call): median wall ms of 5 calls after a warm-up, and the matrix bytes the
call moves over PCIe.  python tools/compat_cost.py > gpurun_out/compat_cost.txt"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))

import numpy as np  # noqa: E402

import gpscore  # noqa: E402
from gpscore import compat  # noqa: E402


def med(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(ts))


print("%6s %-34s %10s %12s" % ("n", "call", "ms", "PCIe MB"))
for n in (500, 2000, 5000):
    d, nt = 8, n // 4
    rng = np.random.default_rng(n)
    X, Xt = rng.standard_normal((n, d)), rng.standard_normal((nt, d))
    y = np.sin(X.sum(1))[:, None]
    a, b, s2 = np.log(1.0), np.log(1.5) * np.ones(d), 0.01
    compat.state.para_k, compat.state.para_l, compat.state.sigma_noise_sq = a, b, s2
    K = compat.ARD(X, X, a, b)
    A = K + s2 * np.eye(n)
    Ksf, Kss = compat.ARD(Xt, X, a, b), compat.ARD(Xt, Xt, a, b)
    mb = lambda *shapes: sum(8.0 * r * c for r, c in shapes) / 1e6  # noqa: E731
    rows = [
        ("compat.ARD(X, X)", lambda: compat.ARD(X, X, a, b), mb((n, n))),
        ("compat.chol_solve(y, A)", lambda: compat.chol_solve(y, A), mb((n, n), (n, 1), (n, 1))),
        ("compat.half_logdet(A)", lambda: compat.half_logdet(A), mb((n, n), (n, n))),
        ("compat.cal_mean_and_cov", lambda: compat.cal_mean_and_cov(Ksf, K, Kss, nt, n, y),
         mb((nt, n), (n, n), (nt, nt)) * 2),
    ]
    gp = gpscore.GP()
    gp.set_data(X, y.ravel())
    gp.set_test(Xt)
    th = (a, b, np.log(s2))
    rows.append(("GP.fit + predict (resident)", lambda: (gp.fit(theta=th, return_loo=False),
                                                         gp.predict()), mb((nt, 1), (nt, 1))))
    for name, fn, m in rows:
        print("%6d %-34s %10.3f %12.1f" % (n, name, med(fn), m), flush=True)
