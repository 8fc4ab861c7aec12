"""The row-sharded FITC path over a REAL RCCL communicator with 2 and 3 ranks, on a one-GPU box
(K20:222-234, 270-296, 236/344/452).

RCCL refuses two ranks on one device ("Duplicate GPU detected"); each rank process here
(tests/rccl_rank.py) presents its own NCCL_HOSTID, so the check passes and the ranks exchange
over the socket transport on loopback instead of xGMI — the same ncclCommInitRank, the same
ncclAllReduce calls on the same streams in the same order as on an 8-GPU node, only slower
links.  Each rank reports what its communicator holds (gps_comm_info: RCCL's ncclCommCount /
ncclCommUserRank), and the gathered shards must match the unsharded fit within 30× the measured
conditioning floor, as the in-process shards of test_gpu_shards do.
"""
import os
import signal
import socket
import subprocess
import sys

import numpy as np
import pytest

from test_gpu_shards import _blockloo_check, _case, _compare, _floor, _whole

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rccl_ranks(P, outdir, args, timeout=240, raw=False):
    port = str(_free_port())
    procs = []
    for r in range(P):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(P),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, NCCL_HOSTID=f"gpscore-test-rank-{r}",
                   NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "rccl_rank.py"), str(outdir)]
                                      + [str(a) for a in args], env=env, start_new_session=True))
    codes = []
    try:
        for p in procs:
            codes.append(p.wait(timeout=timeout))
    finally:
        for p in procs:  # (a rank left inside a collective: end its whole session)
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    assert codes == [0] * P, codes
    if raw:
        return [dict(np.load(os.path.join(outdir, f"rank{r}.npz"))) for r in range(P)]
    parts = []
    for r in range(P):
        z = np.load(os.path.join(outdir, f"rank{r}.npz"))
        part = {"comm": z["comm"].tolist(), "kind": str(z["kind"]),
                "obj": dict(zip(z["obj_keys"].tolist(), z["obj"].tolist())),
                "sc": dict(zip(z["sc_keys"].tolist(), z["sc"].tolist()))}
        for k in z.files:
            if k not in ("comm", "kind", "obj_keys", "obj", "sc_keys", "sc"):
                part[k] = z[k]
        parts.append(part)
    return parts


@pytest.mark.parametrize("P", [2, 3])
def test_fitc_rccl_ranks_match_unsharded(gpu_ctx, tmp_path, P):
    """n = 6001 (ragged shards), m = 300, d = 8: forward, predict, scores and the θ / Z gradients
    of all three objectives over RCCL, each within 30× its measured conditioning floor; every
    rank's communicator counts P ranks and the user ranks are 0..P−1."""
    args = (6001, 1501, 300, 8, 41)
    parts = _rccl_ranks(P, tmp_path, args)
    for r, p in enumerate(parts):
        assert p["comm"] == [P, r] and p["kind"] == "rccl", (p["comm"], p["kind"])
    X, y, Xt, yt, Z, th = _case(*args)
    ref = _whole(X, y, Xt, yt, Z, th, True, gpu_ctx)
    from test_gpu_parity import fitc_cap
    _compare(parts, ref, _floor(X, y, Xt, yt, Z, th, True, gpu_ctx, ref), fitc_cap(Z, th),
             f"fitc_rccl_P{P}")


@pytest.mark.parametrize("P,nfold,objective", [(2, 4, "kc"), (3, 6, "dss")])
def test_fitc_blockloo_rccl_ranks(gpu_ctx, tmp_path, P, nfold, objective):
    """FITC block-LOO with the rows sharded on fold boundaries over RCCL (the other ranks' Σ S_g in
    one m×m all-reduce, the fold values and the gradient's n-sums): every rank returns the
    unsharded value, fold values and θ- / Z-gradients within 30× the measured floor."""
    args = (4000, 10, 40, 4, 45 + P)
    raw = _rccl_ranks(P, tmp_path, args + ("block", nfold, objective), raw=True)
    for r, z in enumerate(raw):
        assert z["comm"].tolist() == [P, r] and str(z["kind"]) == "rccl"
    parts = [(float(z["value"]), z["grad"], z["folds"], z["grad_Z"]) for z in raw]
    X, y, _, _, Z, th = _case(*args)
    _blockloo_check(gpu_ctx, X, y, Z, th, nfold, objective, parts,
                    f"fitc_blockloo_rccl_P{P}_{objective}")


def test_c5_full_size_rccl_two_ranks_bench_line(tmp_path):
    """BASELINE configs[4] (FITC n = 200 000, m = 4000, d = 16) at full size,
    rows sharded over 2 REAL RCCL ranks on the one GPU, through the bench's own N > 1 path
    (`bench.py --gpus 2 --one-gpu-rccl`: the launcher, gps_comm_init, B's chunked ncclAllReduce
    beside the SYRK, the scalar all-reduces).  The line must carry RCCL's own rank counts agreeing
    on both ranks, the sharded C5 outputs equal to the committed N = 1 fixture
    (tests/golden/c5_n1_outputs.json) within its stated tolerance, the RCCL each rank ran, and
    the scaling split (replicated / sharded / exposed exchange, B's bytes and bus rate)."""
    import json
    root = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--one-gpu-rccl",
                        "--config", "C2", "--steps", "1", "--warmup", "1", "--no-grad", "--no-block",
                        "--no-cpu"], env=env, capture_output=True, text=True, timeout=600,
                       start_new_session=True)
    lines = [json.loads(s) for s in p.stdout.splitlines() if s.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, (p.returncode, p.stderr[-3000:])
    j = lines[0]
    f = j["fitc"]
    assert f["rccl"]["all_ranks_agree"] and f["rccl"]["ranks_seen"] == [2], f["rccl"]
    assert f["rccl"]["library"]["all_ranks_same"], f["rccl"]["library"]
    c5 = f["C5"]
    assert c5["config"]["ranks"] == 2 and c5["config"]["n"] == 200000
    par = c5["parity_vs_n1"]
    assert par["ok"] and par["max_err"] <= par["tol"], par
    sp = c5["scaling_split"]
    assert len(sp["per_rank"]) == 2
    for one in sp["per_rank"]:
        ab = one["allreduce_B"]
        # B lower-packed m(m+1)/2 + b (m_pad) + 2 scalars, 8 bytes each, per unit
        assert ab["bytes"] == 8.0 * (4000 * 4001 // 2 + 4096 + 2), ab
        assert ab["bus_GBps"] and ab["bus_GBps"] > 0
        assert one["replicated_ms"] > 0 and one["sharded_ms"] > 0
    with open(os.path.join(str(tmp_path), "c5_rccl2.json"), "w") as fh:
        json.dump(j, fh)
