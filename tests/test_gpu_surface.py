"""contour-plot.R objective surfaces on the GPU (gps_full_surface).

Goldens: tests/golden/make_goldens.py composes CP.R:43-85 from the reference's own Python defs
(rbf SD:8-21 with b = 2·log l, chol_solve KF:25-29, crps KF:60-68, logs KF:52-57) on CP.R's
50 × 50 grid at n = 20 and on a d = 2, n = 100 grid.  R is absent, so R parity is unpinned;
the data are numpy draws of CP.R's generator.  Tolerances: the whole surface normwise, against
the movement a 1e-15 relative perturbation of x causes (measured here on the GPU).
"""
import numpy as np
import pytest

from conftest import load_golden, nrel, record_floors

pytestmark = pytest.mark.gpu

NAMES = ("loo_crps", "insample_crps", "nlml", "loo_logs")


@pytest.mark.parametrize("name", ["surface_cp", "surface_d2"])
def test_surface_vs_golden(gpu_ctx, name):
    import gpscore
    g = load_golden(name)
    got = gpscore.surface(g["x"], g["y"], g["ell"], g["sd"], ctx=gpu_ctx)
    rng = np.random.default_rng(3)
    xp = g["x"] * (1 + 1e-15 * rng.standard_normal(g["x"].shape))
    pert = gpscore.surface(xp, g["y"], g["ell"], g["sd"], ctx=gpu_ctx)
    errs, floors = {}, {}
    for k, nm in enumerate(NAMES):
        errs[nm] = nrel(got[nm], g["surf"][k])
        floors[nm] = nrel(pert[nm], got[nm])
    # absolute ceiling: n ≤ 100 points with σ ≥ the grid's smallest s, cond(A) ≤ n·sf²/s²_min
    cap = 50.0 * len(g["x"]) / float(np.min(g["sd"])) ** 2 * np.finfo(np.float64).eps + 1e-12
    record_floors(name, errs, floors, {nm: cap for nm in NAMES})
    for nm in NAMES:
        err, floor = errs[nm], floors[nm]
        print(f"{name} {nm:14s} gpu-vs-golden {err:.2e}  floor {floor:.2e}  cap {cap:.2e}")
        assert np.all(np.isfinite(got[nm]))
        assert err <= 30 * floor + 1e-12, (nm, err, floor)
        assert max(err, floor) <= cap, (nm, err, floor, cap)


def test_surface_matches_single_point_fits(gpu_ctx):
    """Each grid point is the full-GP fit at that (ℓ, s): the LOO objectives and NLML equal
    gps_full_fit's at θ = (log sf², log ℓ, log s²) (the LOO-LogS without CP.R:81's + s²)."""
    import gpscore
    g = load_golden("surface_d2")
    out = gpscore.surface(g["x"], g["y"], g["ell"], g["sd"], log_sf2=0.3, logs_add_noise=False,
                          ctx=gpu_ctx)
    gp = gpscore.GP(ctx=gpu_ctx)
    for i, sd in enumerate(g["sd"]):
        for j, ell in enumerate(g["ell"]):
            r = gp.fit(g["x"], g["y"], (0.3, np.log(ell), np.log(sd * sd)))
            for k in ("loo_crps", "nlml", "loo_logs"):
                assert abs(out[k][i, j] - r[k]) <= 1e-10 * max(1.0, abs(r[k])), (k, i, j)


def test_surface_edge_cases(gpu_ctx):
    """n = 1, n = 128 (the LDS limit), a non-PD grid point (duplicate inputs, s = 0) → NaN
    there only."""
    import gpscore
    import gp_oracle as O
    x1, y1 = np.array([[0.3]]), np.array([0.7])
    s = gpscore.surface(x1, y1, [0.5, 1.0], [0.1, 0.2], ctx=gpu_ctx)
    ref = O.cp_surface(x1, y1, [0.5, 1.0], [0.1, 0.2])
    for k, nm in enumerate(NAMES):
        assert nrel(s[nm], ref[k]) < 1e-13
    rng = np.random.default_rng(1)
    x = rng.uniform(-4, 4, (128, 3))
    y = np.cos(x.sum(1))
    s = gpscore.surface(x, y, [0.8, 1.5], [0.1, 0.3], ctx=gpu_ctx)
    ref = O.cp_surface(x, y, [0.8, 1.5], [0.1, 0.3])
    for k, nm in enumerate(NAMES):
        assert nrel(s[nm], ref[k]) < 1e-9, (nm, nrel(s[nm], ref[k]))
    xd = np.array([[0.0], [0.0], [1.0]])
    s = gpscore.surface(xd, np.array([1.0, 1.0, 0.0]), [1.0], [0.0, 0.1], ctx=gpu_ctx)
    assert np.all(np.isnan(s["nlml"][0])) and np.all(np.isfinite(s["nlml"][1]))


@pytest.mark.parametrize("n", [129, 700])
def test_surface_beyond_one_wavefront(gpu_ctx, n):
    """n > 128 (past one wavefront's LDS): each grid point runs the resident full-GP path
    (gps_full_fit's factorisation and LOO sums, the in-sample CRPS and CP.R:81's LogS from α and
    diag(A⁻¹)); against the oracle's CP.R objectives, a non-PD point (s = 0 with duplicate
    inputs) NaN there only, and the data left as the context's resident full-GP data."""
    import gpscore
    import gp_oracle as O
    rng = np.random.default_rng(n)
    x = rng.uniform(-4, 4, (n, 2))
    y = np.cos(x.sum(1)) + 0.1 * rng.standard_normal(n)
    ell, sd = [0.6, 1.4, 2.5], [0.05, 0.3]
    s = gpscore.surface(x, y, ell, sd, ctx=gpu_ctx)
    for flag in (True, False):
        s = gpscore.surface(x, y, ell, sd, logs_add_noise=flag, ctx=gpu_ctx)
        ref = O.cp_surface(x, y, ell, sd, logs_add_noise=flag)
        for k, nm in enumerate(NAMES):
            assert nrel(s[nm], ref[k]) < 1e-9, (nm, flag, nrel(s[nm], ref[k]))
    # rows 0 and 1 identical: with s = 0 the second pivot is exactly 1 − 1·1 = 0 (not PD)
    xd = np.vstack([x[:1], x[:1], x[2:]])
    s = gpscore.surface(xd, y, [1.0], [0.0, 0.1], ctx=gpu_ctx)
    assert np.all(np.isnan(s["nlml"][0])) and np.all(np.isfinite(s["nlml"][1]))
    # the surface's data are the context's resident full-GP data now (a fit through the C-ABI
    # without a new gps_full_set_data)
    from gpscore._lib import GPS_ARD, ptr
    th = np.array([0.0, np.log(1.0), np.log(0.01)])
    obj = np.zeros(5)
    gpu_ctx.call("gps_full_fit", GPS_ARD, ptr(th), 1, ptr(obj), None, None)
    f = O.fast_full_fit(xd, y, 0.0, np.log(1.0), np.log(0.01))
    assert abs(obj[0] - f["nlml"]) < 1e-9 * abs(f["nlml"])


def test_surface_concurrent_contexts():
    """Two host threads, each with its own context, call gps_full_surface at n = 128 (the
    133 KB dynamic-LDS configuration) at the same time: the per-device launch attribute is set
    once under a lock, so both grids match the single-threaded result bitwise."""
    from concurrent.futures import ThreadPoolExecutor

    import gpscore
    rng = np.random.default_rng(21)
    x = rng.uniform(-3, 3, (128, 2))
    y = np.sin(x.sum(1))
    ell, sd = np.linspace(0.5, 2.0, 7), np.linspace(0.05, 0.5, 5)

    def job(_):
        ctx = gpscore.Context(0)
        try:
            return [gpscore.surface(x, y, ell, sd, ctx=ctx) for _ in range(3)]
        finally:
            ctx.close()

    with ThreadPoolExecutor(max_workers=2) as ex:
        runs = [r for rs in ex.map(job, range(2)) for r in rs]
    ref = job(0)[0]
    for r in runs:
        for nm in NAMES:
            assert np.array_equal(r[nm], ref[nm]), nm
            assert np.all(np.isfinite(r[nm]))
