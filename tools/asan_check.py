"""Host-side AddressSanitizer pass over the C-ABI: run by tests/test_asan.py in
a subprocess with the ASan runtime first in LD_PRELOAD and GPSCORE_LIB pointing at
libgpscore_asan.so (built by `make asan`, host code instrumented, device code unchanged).

  python tools/asan_check.py null    every entry point with a NULL context (no GPU needed),
                                     gps_ctx_create without a device, gps_last_error(NULL)
  python tools/asan_check.py device  a real context: invalid arguments to every entry point
                                     (each must return < 0 with a message), then small valid
                                     calls through the buffer management paths
Exit status 0 = every check passed and ASan reported nothing (it aborts the process if it does).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd"))

import numpy as np  # noqa: E402

from gpscore import _lib  # noqa: E402


def dummy_args(argtypes):
    out = []
    for t in argtypes:
        if t in (_lib._c_int, _lib._c_i64, ctypes.c_longlong):
            out.append(0)
        elif t is _lib._c_dbl:
            out.append(0.0)
        else:
            out.append(None)
    return out


def null_mode(lib):
    assert lib.gps_version() >= 100
    n = 0
    for name, (_, args) in _lib.SIGNATURES.items():
        if not args or args[0] is not _lib._c_vp or name in ("gps_ctx_destroy", "gps_ctx_stream",
                                                              "gps_last_error"):
            continue
        rc = getattr(lib, name)(*dummy_args(args))
        assert rc == -1, (name, rc)
        assert b"NULL" in lib.gps_last_error(None), name
        n += 1
    assert lib.gps_ctx_destroy(None) == 0 and lib.gps_ctx_stream(None) is None
    h = ctypes.c_void_p()
    rc = lib.gps_ctx_create(0, ctypes.byref(h))
    if rc != 0:  # no device here: the error path, with a message
        assert rc < 0 and len(lib.gps_last_error(None)) > 0
    else:
        lib.gps_ctx_destroy(h)
    print(f"null mode: {n} entry points rejected a NULL context")


def device_mode(lib):
    import gpscore
    ctx = gpscore.Context(0)
    h = ctx.h
    P = _lib.ptr
    X = np.random.default_rng(0).standard_normal((300, 3))
    y = np.sin(X.sum(1))
    th = np.array([0.0, 0.0, np.log(0.05)])
    obj = np.zeros(5)
    bad = [
        ("gps_gram", (h, 7, P(X), 300, P(X), 300, 3, 0.0, P(th), 1, 0.0, 0, P(np.zeros((300, 300))))),
        ("gps_gram", (h, 0, P(X), 0, P(X), 300, 3, 0.0, P(th), 1, 0.0, 0, P(np.zeros(1)))),
        ("gps_gram", (h, 0, P(X), 300, P(X), 200, 3, 0.0, P(th), 1, 0.0, 1, P(np.zeros((300, 200))))),
        ("gps_potrf", (h, 0, None, 0, None)),
        ("gps_potrs", (h, 10, 0, P(np.eye(10)), 10, None, 1, None, 1)),
        ("gps_gemm", (h, 0, 0, 4, 4, 4, 1.0, P(np.eye(4)), 2, P(np.eye(4)), 4, 0.0, P(np.eye(4)), 4)),
        ("gps_scores", (h, None, None, None, 0, 0.0, 1.0, None)),
        ("gps_full_set_data", (h, P(X), P(y), 1, 3)),
        ("gps_full_set_data", (h, P(X), P(y), 300, 0)),
        ("gps_full_set_data", (h, P(X), P(y), 300, 65)),
        ("gps_full_fit", (h, 0, P(th), 1, P(obj), None, None)),  # no data yet
        ("gps_full_predict", (h, None, None, None)),
        ("gps_fitc_set_data", (h, P(X), P(y), 0, 3, 0.0, 1.0, 0)),
        ("gps_fitc_fit", (h, P(th), 1, P(obj), None, None)),
        ("gps_ctx_set_option", (h, 99, 1)),
        ("gps_full_surface", (h, P(X), P(y), 300, 3, 0.0, P(th), 0, P(th), 1, 0, P(np.zeros(4)))),
        ("gps_full_surface", (h, P(X), P(y), 10, 3, 0.0, P(th), 1, P(th), 1, 8, P(np.zeros(4)))),
        ("gps_comm_init", (h, 0, 0, None)),
        ("gps_comm_init_local", (h, 2, 5, 1)),
        ("gps_energy_score", (h, None, None, 0, None, 1, 1.0, None, None)),
    ]
    for name, args in bad:
        rc = getattr(lib, name)(*args)
        assert rc < 0, (name, rc)
        assert len(lib.gps_last_error(h)) > 0, name
    # argument errors after data exist: kind / n_ell / objective / nfold
    ctx.call("gps_full_set_data", P(X), P(y), 300, 3)
    for name, args in [("gps_full_fit", (h, 5, P(th), 1, P(obj), None, None)),
                       ("gps_full_fit", (h, 0, P(th), 2, P(obj), None, None)),
                       ("gps_full_grad", (h, 0, P(th), 1, 9, P(obj), P(np.zeros(3)))),
                       ("gps_full_blockloo", (h, 0, P(th), 1, 0, 0, P(obj), None, None)),
                       ("gps_full_blockloo", (h, 0, P(th), 1, 4, 2, P(obj), None, None))]:
        rc = getattr(lib, name)(*args)
        assert rc < 0, (name, rc)
    # valid calls through the allocation / upload / download paths
    gp = gpscore.GP(ctx=ctx)
    r = gp.fit(X, y, (0.0, 0.0, np.log(0.05)))
    gp.predict(X[:50], y[:50], with_scores=True)
    gp.value_and_grad((0.0, 0.0, np.log(0.05)), "loo_crps")
    gp.block_loo((0.0, 0.0, np.log(0.05)), "kc", grad=True)
    fg = gpscore.GP(ctx=ctx)
    fg.fit(X, y, (0.0, 0.0, np.log(0.05)), kind="fitc", Z=X[:30])
    fg.predict(X[:40], y[:40], with_scores=True)
    fg.value_and_grad((0.0, 0.0, np.log(0.05)), "nlml")
    from gpscore import compat
    compat.chol_solve(np.ones((40, 2)), np.eye(40) * 2.0)
    gpscore.surface(X[:20], y[:20], [0.5, 1.0], [0.1, 0.2], ctx=ctx)
    assert np.isfinite(r["nlml"])
    ctx.close()
    print(f"device mode: {len(bad) + 5} invalid calls rejected, valid paths clean")


if __name__ == "__main__":
    lib = _lib.load()
    assert "asan" in os.path.basename(_lib.LIB_PATH), _lib.LIB_PATH
    (null_mode if sys.argv[1] == "null" else device_mode)(lib)
