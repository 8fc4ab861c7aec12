"""Host-side logic on CPU: theta packing, row sharding, error mapping, and the
multi-rank FITC decomposition exercised with torch.distributed gloo at
world_size 2 (the oracle stands in for the device so the test checks the
sharding / reduction logic, not the kernels)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import gp_oracle as O
from conftest import load_golden, nrel


def test_pack_theta():
    from gpscore.gp import pack_theta
    t, n_ell = pack_theta((0.5, np.array([1.0, 2.0, 3.0]), -1.0), 3)
    assert n_ell == 3 and t.tolist() == [0.5, 1.0, 2.0, 3.0, -1.0]
    t, n_ell = pack_theta((0.5, 0.7, -1.0), 8)
    assert n_ell == 1 and t.tolist() == [0.5, 0.7, -1.0]
    with pytest.raises(ValueError):
        pack_theta((0.5, np.zeros(4), -1.0), 3)


@pytest.mark.parametrize("n,p", [(10, 3), (200000, 8), (7, 8), (40000, 1), (5, 2)])
def test_shard_rows_partition(n, p):
    from gpscore.dist import shard_rows
    spans = [shard_rows(n, p, r) for r in range(p)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c and b >= a
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1
    assert spans == O.shard_bounds(n, p)


@pytest.mark.parametrize("n,k,p", [(4001, 4, 2), (40000, 4, 4), (6001, 6, 3), (1003, 64, 8),
                                   (10, 4, 1)])
def test_fold_shard_rows_nest_folds(n, k, p):
    """Shards on fold boundaries (the sharded FITC block-LOO): a partition of the rows in which
    every fold [int(f·n/k), int((f+1)·n/k)) (KF:496-499) lies inside one shard."""
    from gpscore.dist import fold_shard_rows
    spans = [fold_shard_rows(n, k, p, r) for r in range(p)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c and b > a
    bounds = [n if f == k else int(f * n / k) for f in range(k + 1)]
    for a, b in spans:
        assert a in bounds and b in bounds
    with pytest.raises(ValueError):
        fold_shard_rows(n, k, k + 1, 0)


def test_errors_are_runtime_errors():
    from gpscore import GpsError, NotPositiveDefinite
    assert issubclass(NotPositiveDefinite, RuntimeError)  # caught as in KF:726, K20:784
    assert issubclass(GpsError, RuntimeError)
    e = NotPositiveDefinite(7, "x")
    assert e.info == 7


def test_compat_state_names():
    from gpscore import compat
    for k in ("para_k", "para_l", "sigma_noise_sq", "dtype"):
        assert hasattr(compat.state, k)
    for f in ("ARD", "rbf", "chol_solve", "Q", "cal_mean_and_cov", "spgp_cal_mean_and_cov",
              "crps", "logs", "trivial_loss", "SMSE"):
        assert callable(getattr(compat, f))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, name, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpscore.dist import broadcast_unique_id, global_target_stats, shard_rows
    g = load_golden(name)
    X, y, Z = g["X"], g["y"], g["Z"]
    th = (float(g["log_sf2"]), g["log_ell"], float(g["log_sn2"]))
    a, b = shard_rows(len(y), world, rank)
    # global target statistics (trivial_loss / SMSE inputs) via all-reduce
    mean, var, n_tot = global_target_stats(y[a:b])
    # unique-id broadcast
    uid = broadcast_unique_id(b"\x01" * 128 if rank == 0 else None)
    # the FITC decomposition: local partials -> one all-reduce -> redundant m×m finish
    Kmm, Lm_inv, logdet_m = O.fitc_shared(Z, th[0], th[1])
    part = O.fitc_partials(X[a:b], y[a:b], Z, Lm_inv, *th)
    m = Z.shape[0]
    flat = torch.from_numpy(np.concatenate([part["B"].ravel(), part["b"], part["s"]]))
    dist.all_reduce(flat)
    flat = flat.numpy()
    B, bv, s = flat[:m * m].reshape(m, m), flat[m * m:m * m + m], flat[m * m + m:]
    Lb_inv, logdet_b, c = O.fitc_finish_shared(Kmm, B, bv)
    mu, var_loo = O.fitc_loo_terms(part, y[a:b], Lb_inv, c)
    sums = torch.tensor([np.sum(O.crps_terms(mu, var_loo, y[a:b])),
                         np.sum(O.logs_terms(mu, var_loo, y[a:b]))], dtype=torch.float64)
    dist.all_reduce(sums)
    n = len(y)
    logdet = s[0] + logdet_b - logdet_m
    quad = s[1] - bv @ c
    res = dict(mean=mean, var=var, n_tot=n_tot, uid_ok=uid == b"\x01" * 128,
               nlml=0.5 * n * O.LOG2PI + 0.5 * logdet + 0.5 * quad,
               loo_crps=float(sums[0]) / n, loo_logs=float(sums[1]) / n, a=a, b=b)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), mu=mu, var_loo=var_loo,
             **{k: np.asarray(v) for k, v in res.items()})
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["fitc_n500_m20_rows", "fitc_n2000_m200_rows"])
def test_fitc_gloo_world2(tmp_path, name):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), name, str(tmp_path)), nprocs=world, join=True)
    g = load_golden(name)
    rs = [dict(np.load(tmp_path / f"r{r}.npz")) for r in range(world)]
    mu = np.concatenate([r["mu"] for r in rs])
    var = np.concatenate([r["var_loo"] for r in rs])
    assert nrel(mu, g["loo_mu"]) < 1e-8 and nrel(var, g["loo_var"]) < 1e-8
    for r in rs:
        assert bool(r["uid_ok"])
        assert int(r["n_tot"]) == len(g["y"])
        assert abs(float(r["mean"]) - g["y"].mean()) < 1e-13
        assert abs(float(r["var"]) - g["y"].var(ddof=1)) < 1e-12
        for k in ("nlml", "loo_crps", "loo_logs"):
            assert abs(float(r[k]) - float(g[k])) <= 1e-8 * max(1, abs(float(g[k]))), k


def test_compat_empty_inputs_follow_torch():
    """Empty sides: the reference's ARD is an n×m product (KF:15-21), so an empty side gives
    an empty matrix; crps / logs / MSLL / SMSE are means over the points (KF:52-68, 110-134),
    which torch evaluates to NaN over no points.  Neither reaches the device."""
    from gpscore import compat
    x = np.zeros((0, 3))
    xp = np.ones((4, 3))
    assert compat.ARD(x, xp, 0.0, np.zeros(3)).shape == (0, 4)
    assert compat.rbf(xp, x, 0.0, 0.0).shape == (4, 0)
    e = np.zeros(0)
    assert np.isnan(compat.crps(e, e, e)) and np.isnan(compat.logs(e, e, e))
    assert np.isnan(compat.trivial_loss(e, e, e, np.ones(3)))
    assert np.isnan(compat.SMSE(e, e, np.ones(3)))


def _stats_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpscore.dist import ShardedFITC, global_target_stats, shard_rows
    rng = np.random.default_rng(3)
    y = 1e8 + rng.standard_normal(1001)  # mean far above the spread
    a, b = shard_rows(len(y), world, rank)
    mean, var, n = global_target_stats(y[a:b])

    class _StubGP:  # a communicator already attached: no library call before the check
        comm = (world, rank)

    raised = False
    try:
        ShardedFITC(_StubGP()).set_data(np.zeros((world - 1, 2)), np.zeros(world - 1), None)
    except ValueError:
        raised = True
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), mean=mean, var=var, n=n, raised=raised)
    dist.destroy_process_group()


def test_target_stats_and_empty_shards_world2(tmp_path):
    """global_target_stats is two-pass (a 1e8 offset does not cancel the variance away), and
    fewer training rows than ranks raises on EVERY rank before any shard reaches the library
    (an empty shard used to leave the other ranks waiting in the all-reduce)."""
    world = 2
    mp.spawn(_stats_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    y = 1e8 + np.random.default_rng(3).standard_normal(1001)
    for r in range(world):
        z = np.load(tmp_path / f"s{r}.npz")
        assert abs(float(z["mean"]) - y.mean()) < 1e-7
        assert abs(float(z["var"]) - y.var(ddof=1)) < 1e-9 * y.var(ddof=1)
        assert int(z["n"]) == y.size and bool(z["raised"])
