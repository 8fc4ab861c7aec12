"""Gram builds under every GPS_OPT_GRAM_REG mode given (default 1 2 3) against the oracle and
against mode 1, for d in {8, 16}, full and lower (with the diagonal add), ragged and large
shapes: prints the normwise differences (a quick check for kernel variants before the tests)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))
import gpscore  # noqa: E402
import gp_oracle as O  # noqa: E402
from gpscore._lib import GPS_ARD, ptr  # noqa: E402

modes = [int(a) for a in sys.argv[1:]] or [1, 2, 3]
ctx = gpscore.Context(0)
worst = 0.0
for d in (8, 16):
    for n, m, uplo in ((333, 201, 0), (640, 640, 1), (9000, 4096, 0), (11648, 11648, 1), (5000, 20000, 0)):
        rng = np.random.default_rng(n + m + d)
        x = rng.standard_normal((n, d))
        xp = x if uplo else rng.standard_normal((m, d))
        ell = np.ascontiguousarray(rng.standard_normal(d) * 0.2)
        outs = {}
        for mode in modes:
            ctx.set_gram_reg(mode)
            out = np.full((n, m), -7.0)
            ctx.call("gps_gram", GPS_ARD, ptr(x), n, ptr(xp), m, d, 0.3, ptr(ell), d, 0.01, uplo, ptr(out))
            outs[mode] = np.tril(out) if uplo else out
        rows = rng.choice(n, 64, replace=False)
        ref = O.fast_gram(x[rows], xp, 0.3, ell)
        ref[np.arange(64)[rows < m], rows[rows < m]] += 0.01
        if uplo:
            ref = np.where(np.arange(m)[None, :] <= rows[:, None], ref, 0.0)
        for mode, out in outs.items():
            e = np.linalg.norm(out[rows] - ref) / np.linalg.norm(ref)
            e1 = np.linalg.norm(out - outs[modes[0]]) / np.linalg.norm(outs[modes[0]])
            worst = max(worst, e)
            print(f"d={d} n={n} m={m} uplo={uplo} mode={mode}: vs oracle {e:.2e}  vs mode {modes[0]} {e1:.2e}")
ctx.set_gram_reg(True)
print("worst", worst)
sys.exit(0 if worst < 1e-13 else 1)
