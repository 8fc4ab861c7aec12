"""bench.py's own launcher (VERDICT r3 "next" 1): `python bench.py --gpus N` with no WORLD_SIZE in
the environment starts N rank processes itself, which meet over gloo; a WORLD_SIZE that disagrees
with --gpus is refused; a failing rank makes the whole run fail.  `--dry` stops every rank before
any device call (it loads libgpscore only for gps_rccl_info, which needs no device), so this runs
on the CPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=timeout)


def _json_lines(out):
    return [json.loads(s) for s in out.splitlines() if s.startswith("{")]


def test_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry"])
    assert r.returncode == 0, r.stderr
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    j = lines[0]
    assert j["n_gpus"] == 2 and j["ranks_ok"], j
    assert sorted(x[0] for x in j["ranks"]) == [0, 1]
    assert sorted(x[1] for x in j["ranks"]) == [0, 1]  # LOCAL_RANK = device index
    assert os.getpid() not in [x[2] for x in j["ranks"]]


def test_gpus4_spawns_four_ranks():
    r = _run(["--gpus", "4", "--dry"])
    assert r.returncode == 0, r.stderr
    (j,) = _json_lines(r.stdout)
    assert j["n_gpus"] == 4 and j["ranks_ok"], j


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "1", "--dry"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "refusing" in r.stderr


def test_failing_rank_fails_the_run():
    r = _run(["--gpus", "2", "--dry"], {"GPS_BENCH_DRY_FAIL": "1"})
    assert r.returncode != 0
    assert not _json_lines(r.stdout)


def test_single_gpu_runs_in_process():
    r = _run(["--dry"])
    assert r.returncode == 0, r.stderr
    (j,) = _json_lines(r.stdout)
    assert j["n_gpus"] == 1 and j["ranks"][0][:2] == [0, 0]


def test_dry_reports_communicator_rank_counts():
    """The FITC leg's self-check: every rank's communicator count and user rank
    gathered into fitc.rccl; at --gpus 2 both ranks agree."""
    r = _run(["--gpus", "2", "--dry"])
    assert r.returncode == 0, r.stderr
    (j,) = _json_lines(r.stdout)
    rc = j["fitc"]["rccl"]
    assert rc["ranks_seen"] == [2] and rc["all_ranks_agree"], rc
    assert sorted(p["comm_user_rank"] for p in rc["per_rank"]) == [0, 1]
    assert "failures" not in j


def test_dry_wrong_communicator_count_fails_the_run():
    """A communicator that counts other than --gpus ranks: the line still prints (it carries the
    evidence) and the run exits non-zero."""
    r = _run(["--gpus", "2", "--dry"], {"GPS_BENCH_DRY_COMM_COUNT": "1:1"})
    assert r.returncode == 4, (r.returncode, r.stderr)
    (j,) = _json_lines(r.stdout)
    assert not j["fitc"]["rccl"]["all_ranks_agree"]
    assert j["fitc"]["rccl"]["ranks_seen"] == [1, 2]
    assert j["failures"]


def test_spawner_forwards_sigterm_to_ranks():
    """a SIGTERM to the spawner itself (not to its process group) stops the ranks and
    fails the run instead of orphaning them."""
    import signal
    import time

    import psutil
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MASTER_ADDR="127.0.0.1", GPS_BENCH_DRY_SLEEP="60")
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2", "--dry"], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        parent = psutil.Process(p.pid)
        deadline = time.time() + 60
        kids = []
        while time.time() < deadline and len(kids) < 2:
            kids = parent.children()
            time.sleep(0.2)
        assert len(kids) == 2, kids
        time.sleep(1.0)
        p.send_signal(signal.SIGTERM)
        out, err = p.communicate(timeout=45)
        assert p.returncode == 128 + signal.SIGTERM, (p.returncode, err)
        gone, alive = psutil.wait_procs(kids, timeout=10)
        assert not alive, alive
    finally:
        if p.poll() is None:
            p.kill()


def test_dry_pins_the_scaling_split_schema():
    """the N > 1 line explains its scaling — per rank the replicated, sharded
    and exposed-exchange ms of the FITC unit, B's all-reduce bytes / time / bus rate, and which
    RCCL each rank runs (version and the file holding ncclAllReduce).  --dry builds the split with
    the production code (bench.scaling_split) on a stand-in phase record."""
    r = _run(["--gpus", "2", "--dry"])
    assert r.returncode == 0, r.stderr
    (j,) = _json_lines(r.stdout)
    lib = j["fitc"]["rccl"]["library"]
    assert lib["version"] >= 20000 and "rccl" in os.path.basename(lib["path"]), lib
    assert lib["all_ranks_same"] and lib["why"]
    sp = j["fitc"]["C5"]["scaling_split"]
    assert len(sp["per_rank"]) == 2
    one = sp["per_rank"][0]
    for k in ("replicated_ms", "sharded_ms", "exposed_exchange_ms", "predict_and_rest_ms",
              "phases_ms", "allreduce_B", "allreduce_small"):
        assert k in one, k
    assert one["replicated_ms"] == 3.0 and one["sharded_ms"] == 4.0
    assert one["exposed_exchange_ms"] == 2.0 and one["predict_and_rest_ms"] == 11.0
    ab = one["allreduce_B"]
    assert ab["count"] == 4 and ab["bytes"] == 8.0 * 4000 * 4001 / 2
    # ring bus rate at N = 2: 2(N−1)/N · bytes / time
    assert abs(ab["bus_GBps"] - ab["bytes"] / 4e-3 / 1e9) < 1e-9
    assert sp["max_over_ranks"]["replicated_ms"] == 3.0


def test_scaling_model_classes():
    """bench.scaling_model: the kernel-accounting classes split into replicated (the m×m work every
    rank repeats), sharded and exchange, and the compute projection replicated + sharded·N0/N."""
    sys.path.insert(0, ROOT)
    import bench
    prof = {"potrf_dag": {"count": 4, "ms": 4.0, "flop": 1.0, "bytes": 0},
            "gemm_trmm_l": {"count": 6, "ms": 2.0, "flop": 1.0, "bytes": 0},
            "gemm_rowsq": {"count": 6, "ms": 100.0, "flop": 1.0, "bytes": 0},
            "gemm_syrk_splitk": {"count": 1, "ms": 50.0, "flop": 1.0, "bytes": 0},
            "allreduce_B": {"count": 4, "ms": 1.0, "flop": 0, "bytes": 6.4e7}}
    m = bench.scaling_model(prof, 2, 1)
    assert m["replicated_kernels_ms"] == 3.0 and m["sharded_kernels_ms"] == 75.0
    assert m["exchange_kernels_ms"] == 0.5
    assert m["compute_projection_ms"]["8"] == 3.0 + 75.0 / 8
