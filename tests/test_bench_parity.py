"""bench.py's N > 1 self-check on the CPU: the sharded C5 unit's outputs are
reduced to rank-independent quantities (global objectives and scores, all-rank sums and sampled
entries of the LOO / predictive vectors, gathered over gloo) and compared with the committed
N = 1 fixture.  A stand-in GP serves each rank's rows of fixed vectors, so world 1 and world 2
must report the same quantities, and a perturbed shard must fail the comparison."""
import json
import os
import socket

import numpy as np
import pytest

from conftest import ROOT

import bench


class _FakeFit:
    def __init__(self, obj, mu, var):
        self.objectives, self.mu_loo, self.var_loo = obj, mu, var


class _FakeGP:
    """The rows [a, b) / test rows [ta, tb) of fixed global vectors, as a rank's GP returns them."""

    def __init__(self, full, rows, test_rows, bump=0.0):
        self.full, self.rows, self.test_rows, self.bump = full, rows, test_rows, bump

    def fit(self, theta=None):
        a, b = self.rows
        return _FakeFit(dict(self.full["obj"]), self.full["loo_mu"][a:b] + self.bump,
                        self.full["loo_var"][a:b])

    def predict(self, with_scores=True):
        a, b = self.test_rows
        return self.full["pred_mu"][a:b], self.full["pred_var"][a:b], dict(self.full["sc"])


N, NT = 1000, 300
FC = {"n": N, "nt": NT}


def _full():
    rng = np.random.default_rng(0)
    return {"obj": {"nlml": -1234.5, "loo_crps": 0.07, "loo_logs": -0.8, "logdet": -5e3, "quad": 900.0},
            "sc": {"test_crps": 0.08, "test_logs": -0.7, "test_msll": -2.0, "test_smse": 0.01,
                   "test_mse": 0.02, "test_cover": 0.95},
            "loo_mu": rng.standard_normal(N), "loo_var": rng.random(N) + 0.01,
            "pred_mu": rng.standard_normal(NT), "pred_var": rng.random(NT) + 0.01}


def _outputs_world1():
    ctl = bench.Ctl(1)
    return bench.fitc_outputs(ctl, _FakeGP(_full(), (0, N), (0, NT)), None, FC, (0, N), (0, NT))


def _worker(rank, world, port, out, bump_rank):
    import torch.distributed as dist
    from gpscore.dist import shard_rows
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctl = bench.Ctl.__new__(bench.Ctl)
    ctl.world, ctl.dist = world, dist
    rows, trows = shard_rows(N, world, rank), shard_rows(NT, world, rank)
    gp = _FakeGP(_full(), rows, trows, bump=1e-6 if rank == bump_rank else 0.0)
    res = bench.fitc_outputs(ctl, gp, None, FC, rows, trows)
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _outputs_sharded(tmp_path, world, bump_rank=-1):
    import torch.multiprocessing as mp
    out = str(tmp_path / f"w{world}_{bump_rank}.json")
    mp.spawn(_worker, args=(world, _free_port(), out, bump_rank), nprocs=world, join=True)
    with open(out) as f:
        return json.load(f)


def _fixture(outs):
    return json.loads(json.dumps(dict(outs, tol=1e-9, source="test")))


def test_sample_indices_cover_shard_boundaries():
    from gpscore.dist import shard_rows
    idx = set(bench.sample_indices(200000))
    for p in (2, 4, 8):
        for r in range(1, p):
            a, _ = shard_rows(200000, p, r)
            assert {a - 1, a} <= idx
    assert 0 in idx and 199999 in idx


def test_world1_matches_itself():
    ref = _fixture(_outputs_world1())
    cmp = bench.compare_fitc_outputs(json.loads(json.dumps(_outputs_world1())), ref)
    assert cmp["ok"] and cmp["max_err"] == 0.0, cmp


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_outputs_equal_world1(tmp_path, world):
    ref = _fixture(_outputs_world1())
    got = _outputs_sharded(tmp_path, world)
    cmp = bench.compare_fitc_outputs(got, ref)
    assert cmp["ok"], cmp
    assert cmp["max_err"] < 1e-14, cmp  # only the sums' association differs
    for k in bench.FITC_VECS:
        assert got["vectors"][k]["count"] == ref["vectors"][k]["count"]


def test_perturbed_shard_fails(tmp_path):
    ref = _fixture(_outputs_world1())
    got = _outputs_sharded(tmp_path, 2, bump_rank=1)
    cmp = bench.compare_fitc_outputs(got, ref)
    assert not cmp["ok"] and cmp["worst"].startswith("loo_mu"), cmp


def test_missing_rows_fail_layout():
    ref = _fixture(_outputs_world1())
    ctl = bench.Ctl(1)
    got = bench.fitc_outputs(ctl, _FakeGP(_full(), (0, N - 1), (0, NT)), None, FC, (0, N - 1),
                             (0, NT))
    cmp = bench.compare_fitc_outputs(json.loads(json.dumps(got)), ref)
    assert not cmp["ok"] and cmp["max_err"] == float("inf")


def test_committed_c5_fixture_is_well_formed():
    path = bench.C5_FIXTURE
    if not os.path.exists(path):
        pytest.skip("C5 fixture not generated yet (bench.py --write-c5-fixture on the GPU box)")
    with open(path) as f:
        fx = json.load(f)
    assert fx["config"]["n"] == 200000 and fx["config"]["m"] == 4000
    assert 0 < fx["tol"] < 1e-7
    for k in bench.FITC_VECS:
        v = fx["vectors"][k]
        assert v["count"] == (200000 if k.startswith("loo") else 10000)
        assert set(int(i) for i in v["samples"]) == set(bench.sample_indices(v["count"]))
    assert set(fx["objectives"]) == {"nlml", "loo_crps", "loo_logs", "logdet", "quad"}
    assert os.path.relpath(path, ROOT) == os.path.join("tests", "golden", "c5_n1_outputs.json")
