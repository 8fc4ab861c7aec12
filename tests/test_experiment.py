"""Host logic of the replicate harness (gpscore.experiment): the
scripts' per-replicate row draws (Python's `random`, KF:194-203), the split, the sheet
loaders, and the method table (itr / lr / starts as KF and K20 write them).  No GPU."""
import random

import numpy as np

from gpscore import experiment as E


def test_replicate_indices_are_the_scripts_draws():
    for j in (0, 1, 7):
        random.seed(j * 100)                                            # KF:194
        sam = np.reshape(random.sample(range(0, 10000), 500 + 300), (800,))  # KF:196
        va = np.reshape(random.sample(range(0, 800), 300), (300,))           # KF:203
        s2, v2 = E.replicate_indices(j)
        assert np.array_equal(sam, s2) and np.array_equal(va, v2)


def test_unseeded_stream_continues_across_replicates():
    """K20 never reseeds (K20:184-192): one stream feeds every replicate."""
    rs, ref = random.Random(5), random.Random(5)
    for _ in range(3):
        s, v = E.replicate_indices(None, rs=rs)
        assert np.array_equal(s, ref.sample(range(0, 10000), 800))
        assert np.array_equal(v, ref.sample(range(0, 800), 300))


def test_replicate_split_and_loaders(tmp_path):
    sheets = E.synthetic_sheets(0, n_pool=10000, n_test=600, d=8)
    np.savez(tmp_path / "kin.npz", **sheets)
    csv = tmp_path / "csv"
    csv.mkdir()
    for k, v in sheets.items():
        np.savetxt(csv / f"{k}.csv", v, delimiter=",")
    for loaded in (E.load_sheets(str(tmp_path / "kin.npz")), E.load_sheets(str(csv))):
        assert all(loaded[k].shape == sheets[k].shape for k in E.SHEETS)
        data = E.replicate(loaded, j=2)
        assert data["train_x"].shape == (500, 8) and data["va_x"].shape == (300, 8)
        assert data["test_x"].shape == (500, 8) and data["train_y"].shape == (500,)
        sam, va = E.replicate_indices(2)
        full = loaded["trainx"][sam]
        assert np.array_equal(data["va_x"], full[va])
        assert np.array_equal(data["train_x"], full[np.setdiff1d(np.arange(800), va)])
        assert np.array_equal(data["test_y"], loaded["testy"][:500, 0])


def test_method_tables_follow_the_scripts():
    kf, k20 = E.KF_METHODS, E.K20_METHODS
    assert [(m.itr, m.lr) for m in kf.values()] == [(400, 1.0), (400, 5e-4), (500, 0.05),
                                                    (150, 1e-3), (25, 0.1)]
    assert [(m.itr, m.lr, m.lr_z) for m in k20.values()] == [
        (2000, 1.0, 1.0), (3000, 1e-4, 1e-3), (3000, 0.2, 0.2), (3000, 1e-3, 1e-3),
        (3000, 0.1, 0.1)]
    assert kf["crps"].init == "rand3" and k20["logs"].init == "ones" and k20["dss"].z_init == "randn"
    rng = np.random.default_rng(0)
    k, ell, s = E.initial_theta(kf["crps"], 8, rng)
    assert 0 <= k < 1 and ell.shape == (8,) and 0 <= s < 1
    assert E.initial_theta(k20["logs"], 8, rng)[1].shape == (1,)
