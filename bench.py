#!/usr/bin/env python3
"""Benchmark of the GP hot path on MI355X (BASELINE.json metric).

One step = one "unit" of the reference's per-iteration work at fixed theta:
fit (Gram + Cholesky + L⁻¹ + α + diag(A⁻¹) → NLML, LOO-CRPS, LOO-LogS) + predict
(μ*, σ²* at the test points) + score (CRPS, LogS, MSLL, SMSE, MSE, coverage).

* Headline (``value``): full GP C3 (n = 20 000, d = 8, n* = 5 000), one unit per
  rank per step.  The full GP does not shard (replicas only): under torchrun
  every rank runs its own unit, value = units of all ranks / max-over-ranks time.
* ``fitc``: FITC C5 (n = 200 000, m = 4 000, d = 16, n* = 10 000) with the rows
  sharded over the ranks and ONE RCCL all-reduce of the m×m accumulator (strong
  scaling: fixed total work); at N = 1 also C4 (n = 40 000, m = 2 000, d = 8).
* ``roofline``: the FP64-MFMA GEMM kernel (potrf trailing updates, inverse,
  predictive TRMM) — algorithmic flops / summed kernel time from hipEvents
  recorded on the library's stream over the timed region; ``roofline_gram`` the
  HBM-bound Gram kernel.
* ``cpu_baseline``: the torch-CPU fp64 ref-mirror of the reference op sequence
  (oracle/ref_torch.py, all host threads) timed on one full C3 unit; rank 0 at N = 1
  only.  ``parity``: every output of the GPU unit against that run's outputs (same
  inputs).  ``c1``: BASELINE.json configs[0] (SIMPLE-DATA n = 500, d = 1, rbf) on the
  GPU and on the host.  ``fitc.C4.cpu_baseline``: dense FITC ref-mirror (n³-extrapolated)
  and the Woodbury numpy restatement.

Inputs are synthetic (SURVEY.md §8d generator) and resident in HBM before the
timed region.  Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd")
sys.path.insert(0, PKG_DIR)

METRIC = "GP fit+predict+CRPS wall-clock (ms) at n=20k full / n=40k FITC; HBM GB/s & MFMA%"
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 matrix (= vector) peak, spec
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)

CONFIGS = {
    "C2": dict(n=5000, d=8, nt=1250, seed=2),
    "C3": dict(n=20000, d=8, nt=5000, seed=3),
    "C4": dict(n=40000, d=8, nt=10000, m=2000, seed=4),
    "C5": dict(n=200000, d=16, nt=10000, m=4000, seed=5),
    # one rank's share of C5 at N = 8 / 4 / 2 (rows 25 000 / 50 000 / 100 000): the per-rank unit of
    # the strong-scaling run without the exchange, for single-GPU A/Bs (tools/ab_bench.py)
    "C5r8": dict(n=25000, d=16, nt=1250, m=4000, seed=5),
    "C5r4": dict(n=50000, d=16, nt=2500, m=4000, seed=5),
    "C5r2": dict(n=100000, d=16, nt=5000, m=4000, seed=5),
}


def synth(n, d, nt, seed, m=None):
    """X, Xt ~ N(0, I); y = sin(3 X w) + 0.1 ε; Z = m training rows."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d))
    Xt = rng.standard_normal((nt, d))
    w = rng.standard_normal(d) / np.sqrt(d)
    y = np.sin(3 * X @ w) + 0.1 * rng.standard_normal(n)
    yt = np.sin(3 * Xt @ w) + 0.1 * rng.standard_normal(nt)
    Z = X[rng.choice(n, m, replace=False)] if m else None
    theta = (0.0, np.log(2.0) * np.ones(d), np.log(0.01))
    return X, y, Xt, yt, Z, theta


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, one_gpu_rccl=False):
    """`bench.py --gpus N` without a launcher's WORLD_SIZE: start N rank processes of this same
    script (one per GPU, RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free
    MASTER_PORT) and wait on them.  This parent only spawns and collects: it never imports torch or
    gpscore and never touches the GPU (children are started as new processes, not by exec).  The
    one JSON line comes from rank 0's stdout, which the children share with this process.  If a
    rank fails, the others are terminated and the first non-zero exit status is returned."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    stop = {"sig": None}

    def on_signal(signum, _frame):  # the parent itself told to stop: the ranks go with it
        stop["sig"] = signum
    old_handlers = {sg: signal.signal(sg, on_signal) for sg in (signal.SIGTERM, signal.SIGINT)}
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=port)
        if one_gpu_rccl:  # (--one-gpu-rccl: each rank its own RCCL host id, loopback sockets)
            env.update(NCCL_HOSTID=f"gpscore-rank-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    kill_at = None
    live = list(procs)
    while live:
        if stop["sig"] is not None and kill_at is None:
            print(f"[bench] spawner got signal {stop['sig']}; stopping the ranks", file=sys.stderr,
                  flush=True)
            rc = rc or 128 + stop["sig"]
            for q in live:
                q.send_signal(signal.SIGTERM)
            kill_at = time.time() + 30.0
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"[bench] rank {procs.index(p)} exited with status {code}; stopping the others",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.send_signal(signal.SIGTERM)
                kill_at = time.time() + 30.0  # a rank stuck in a collective may ignore SIGTERM
        if kill_at is not None and time.time() > kill_at:
            for q in live:
                q.kill()
            kill_at = float("inf")
        time.sleep(0.2)
    for sg, h in old_handlers.items():
        signal.signal(sg, h)
    return rc


class Ctl:
    """Control plane: barrier and max-over-ranks (gloo on the host; the data-path
    collective is RCCL inside libgpscore)."""

    def __init__(self, world):
        self.world = world
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo prints a "[Gloo] Rank i is connected ..." banner on fd 1; keep stdout
            # to the one JSON line rank 0 emits
            sys.stdout.flush()
            saved = os.dup(1)
            devnull = os.open(os.devnull, os.O_WRONLY)
            os.dup2(devnull, 1)
            try:
                dist.init_process_group("gloo")
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(devnull)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, v):
        if not self.dist:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

    def gather(self, obj):
        """every rank's `obj`, in rank order, on every rank (gloo object all-gather)"""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out


def sync_all(ctl, ctx):
    ctx.synchronize()
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass
    ctl.barrier()


def timed(ctl, ctx, fn, steps):
    sync_all(ctl, ctx)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync_all(ctl, ctx)
    return ctl.max(time.perf_counter() - t0)


def kernel_pass(ctl, ctx, fn, steps):
    """Time `steps` more steps with every launch bracketed by hipEvents on its own
    (single) stream, so each launch's duration is its own (overlap off)."""
    ctx.set_overlap(False)
    ctx.prof(True)
    t = timed(ctl, ctx, fn, steps)
    prof = ctx.prof_collect()
    ctx.prof(False)
    ctx.set_overlap(True)
    return prof, 1e3 * t / steps


def kernel_summary(prof, steps):
    """per-step kernel stats from the library's hipEvent records."""
    out = {}
    for tag, v in sorted(prof.items()):
        out[tag] = {"count": v["count"] / steps, "ms": v["ms"] / steps,
                    "tflops": (v["flop"] / (v["ms"] * 1e-3) / 1e12) if v["flop"] and v["ms"] else None,
                    "gbs": (v["bytes"] / (v["ms"] * 1e-3) / 1e9) if v["bytes"] and v["ms"] else None}
    return out


TRAFFIC_KIND = ("L2-fabric bytes per launch (rocprofv3 FETCH_SIZE + WRITE_SIZE, gfx950 "
                "corrections; every L2 miss, Infinity-Cache hits included: an upper bound on HBM "
                "bytes), from the committed counter passes (tools/profile_round.sh)")


def alg_flop(kind, c, world=1):
    """BASELINE.md §"Unit and roofline" algorithmic flops of one unit at the UNPADDED sizes:
    full GP n³/3 (potrf) + n³/3 (trtri) + n²·n* (predictive TRMM); FITC 2m³/3 (the two m×m
    factorisations) + 3·n·m² (two row-norm TRMMs, the B SYRK) + 2·n*·m² (predict)."""
    if kind == "full":
        return 2.0 * c["n"] ** 3 / 3.0 + float(c["n"]) ** 2 * c["nt"]
    # per rank: the m×m factorisations are replicated, the row work is sharded
    return 2.0 * c["m"] ** 3 / 3.0 + (3.0 * c["n"] + 2.0 * c["nt"]) * c["m"] ** 2 / world


MFMA_TAGS = ("gemm", "potrf_dag")


def phases(ctl, ctx, model, theta, steps, prof, ms_unit, upload=None):
    """each phase of the unit and their sum — fit (Gram, factor, logdet, α,
    diag A⁻¹ -> NLML / LOO-CRPS / LOO-LogS) and predict (μ*, σ²* and the fused score sums)
    timed separately on the production path; the score kernels' share from the kernel pass.
    `upload` (host -> HBM copies of the inputs) gives the PCIe-inclusive end-to-end figure, which
    is never `value`."""
    up_ms = 1e3 * timed(ctl, ctx, upload, steps) / steps if upload else None
    t_fit = timed(ctl, ctx, lambda: model.fit(theta=theta, return_loo=False), steps)
    t_pred = timed(ctl, ctx, lambda: model.predict(with_scores=True), steps)
    fit_ms, pred_ms = 1e3 * t_fit / steps, 1e3 * t_pred / steps
    sc = prof.get("score_sums", {})
    return {"fit_ms": fit_ms, "predict_ms": pred_ms,
            "score_ms": sc.get("ms", 0.0) / steps if sc else None,
            "sum_ms": fit_ms + pred_ms, "unit_ms": ms_unit, "upload_ms": up_ms,
            "end_to_end_ms": (up_ms + fit_ms + pred_ms) if upload else None,
            "note": "predict_ms includes the score (fused into the predict call: one launch pair "
                    "after the finalise); score_ms = those kernels alone (single-stream pass)"}


def roofline_mfma(prof, traffic=None, steps=1, flop_alg=None):
    """Every MFMA launch of a step — the GEMMs and the persistent factorisation of the bottom
    diagonal blocks, which carries part of the n³/3 + n³/3: achieved = algorithmic flops
    (unpadded, alg_flop) ÷ their summed launch time; the padded flops the launches execute and
    the GEMM launches alone are reported beside."""
    f = sum(v["flop"] for k, v in prof.items() if k.startswith(MFMA_TAGS)) / steps
    ms = sum(v["ms"] for k, v in prof.items() if k.startswith(MFMA_TAGS)) / steps
    n = sum(v["count"] for k, v in prof.items() if k.startswith(MFMA_TAGS)) / steps
    ms_g = sum(v["ms"] for k, v in prof.items() if k.startswith("gemm")) / steps
    f_g = sum(v["flop"] for k, v in prof.items() if k.startswith("gemm")) / steps
    fa = flop_alg if flop_alg is not None else f
    ach = fa / (ms * 1e-3) / 1e12 if ms else 0.0
    return {"bound": "mfma", "kernel": "gemm_f64_kernel + potrf_dag_kernel (every MFMA launch of the step)",
            "gemm_launches_alone": {"ms_per_step": ms_g, "tflops_at_padded_flop":
                                    round(f_g / (ms_g * 1e-3) / 1e12, 3) if ms_g else 0.0},
            "achieved": round(ach, 3), "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / PEAK_FP64_TFLOPS, 4), "traffic": traffic,
            "traffic_kind": TRAFFIC_KIND if traffic is not None else None,
            "launches_per_step": n, "avg_launch_ms": ms / n if n else None,
            "flop_per_launch": fa / n if n else None, "flop_alg_per_step": fa,
            "flop_padded_per_step": f,
            "achieved_at_padded_flop": round(f / (ms * 1e-3) / 1e12, 3) if ms else 0.0}


def roofline_trailing(prof, steps=1):
    """The Cholesky trailing updates A22 -= L21 L21ᵀ alone (the lower-tile SYRK launches of
    the recursion, every size class) — the MFMA-utilisation figure north_star names."""
    ks = [k for k in prof if k.startswith("gemm_syrk")]
    f = sum(prof[k]["flop"] for k in ks) / steps
    ms = sum(prof[k]["ms"] for k in ks) / steps
    n = sum(prof[k]["count"] for k in ks) / steps
    ach = f / (ms * 1e-3) / 1e12 if ms else 0.0
    return {"bound": "mfma", "kernel": "gemm_f64_kernel lower-tile SYRK (trailing updates)",
            "achieved": round(ach, 3), "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / PEAK_FP64_TFLOPS, 4), "launches_per_step": n,
            "ms_per_step": ms, "flop_per_step": f}


def roofline_gram(prof, steps=1, traffic=None, tags=("gram_kff", "gram_ksf")):
    b = sum(prof[t]["bytes"] for t in tags if t in prof) / steps
    ms = sum(prof[t]["ms"] for t in tags if t in prof) / steps
    ach = b / (ms * 1e-3) / 1e9 if ms else 0.0
    return {"bound": "hbm", "kernel": "gram_mfma_kernel<8> (K_ff lower + K*f)", "achieved": round(ach, 1),
            "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4),
            "traffic": traffic, "traffic_kind": TRAFFIC_KIND if traffic is not None else None,
            "bytes_per_step": b,
            "bytes_per_launch": b / max(1, sum(1 for t in tags if t in prof))}


def _oracle():
    for sub in ("oracle",):
        p = os.path.join(ROOT, sub)
        if p not in sys.path:
            sys.path.insert(0, p)
    import gp_oracle as O
    import ref_torch as RT
    return O, RT


def host_cores():
    """The host threads this process may use and how that was decided: the CPU affinity mask
    (os.sched_getaffinity), capped by OMP_NUM_THREADS when the box sets it (the lease's share
    on a shared host; os.cpu_count() reports the whole machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    used = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    return used, {"threads_used": used, "sched_getaffinity": aff, "os_cpu_count": os.cpu_count(),
                  "OMP_NUM_THREADS": omp}


def _torch_threads():
    import torch
    cores, _ = host_cores()
    torch.set_num_threads(cores)
    return cores


def cpu_baseline(config="C3"):
    """The reference op sequence in the reference's own framework — torch-CPU fp64 ref-mirror
    (oracle/ref_torch.py: upper potrf + 2 LU solves per chol_solve, LOO diag by
    chol_solve(I, A), full n*×n* covariance; KF:239-245, 329-334, 365-391) — timed on ONE
    full C3 unit on the box's host threads (BASELINE.md:48-57).  Also returns its outputs,
    which the parity record compares with the GPU unit."""
    O, RT = _oracle()
    cores = _torch_threads()
    _, cinfo = host_cores()
    c = CONFIGS[config]
    X, y, Xt, yt, _, th = synth(c["n"], c["d"], c["nt"], c["seed"])
    t0 = time.perf_counter()
    ref = RT.ref_full(X, y, Xt, yt, *th)
    t = time.perf_counter() - t0
    # BASELINE.md:53's second CPU figure: the numpy/LAPACK potrf + trsm restatement (the GPU's
    # algorithm, oracle.fast_full) on the same unit and the same number of BLAS threads
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=cores):
        t0 = time.perf_counter()
        O.fast_full(X, y, Xt, yt, *th)
        t_fast = time.perf_counter() - t0
    info = RT.host_info()
    info.update(cinfo)
    scaling = cpu_thread_scaling(RT, cores)
    return {"value": 1.0 / t, "unit": f"fit+predict+score units/s ({config})",
            "threads_rationale": "threads_used = the lease's host-CPU share: the GPU box presets "
                                 "OMP_NUM_THREADS to its share of the host (16 per GPU) and its "
                                 "rules size worker pools to that share, while sched_getaffinity / "
                                 "os.cpu_count report the whole 256-thread host; threads beyond "
                                 "the share would run on other jobs' CPUs.  thread_scaling below "
                                 "measures how the ref-mirror scales up to the share.",
            "thread_scaling": scaling,
            "cores": cores, "kind": "port", "host": info,
            "sample": f"torch-CPU fp64 ref-mirror of the reference op sequence on the full C3 "
                      f"workload {config} n={c['n']} d={c['d']} n*={c['nt']}, one unit: {t:.1f} s "
                      f"({info['cpu_model']}, {cores} threads, BLAS {info['blas']})",
            "fast_cpu_s": t_fast,
            "fast_cpu_note": "oracle.fast_full: numpy/LAPACK potrf + L^-1 products on the same unit "
                             f"and {cores} BLAS threads (the GPU's algorithm, not the reference's "
                             "op sequence)"}, ref


def cpu_thread_scaling(RT, cores):
    """The torch-CPU ref-mirror on a quarter-C2 unit (n = 2500, d = 8, n* = 625) at 1, 2, 4, …
    threads up to the lease's share: the parallel efficiency t(1) / (p·t(p)) shows how the
    threads_used baseline would move with more host threads (an estimate beyond p, and a
    conservative one: the C3 unit has 512× this unit's flops to spread)."""
    import torch
    n, nt = 2500, 625
    X, y, Xt, yt, _, th = synth(n, 8, nt, 2)
    out = {}
    p = 1
    while p <= cores:
        torch.set_num_threads(p)
        RT.ref_full(X[:256], y[:256], Xt[:64], yt[:64], *th)  # spin the pool up at this width
        t0 = time.perf_counter()
        RT.ref_full(X, y, Xt, yt, *th)
        out[str(p)] = time.perf_counter() - t0
        p *= 2
    torch.set_num_threads(cores)
    t1 = out["1"]
    return {"workload": f"n={n}, d=8, n*={nt} unit, torch-CPU fp64 ref-mirror",
            "seconds": out,
            "efficiency": {k: t1 / (int(k) * v) for k, v in out.items()}}


PARITY_VECS = ("loo_mu", "loo_var", "pred_mu", "pred_var")
PARITY_SCAL = ("nlml", "loo_crps", "loo_logs", "logdet", "quad", "test_crps", "test_logs",
               "test_msll", "test_smse", "test_mse", "test_cover")


def parity(got, ref):
    """normwise relative error of every output of the unit against the oracle run on the
    same inputs: max|a − b| / max|b| for vectors, |a − b| / max(1, |b|) for scalars."""
    out = {}
    for k in PARITY_VECS:
        a, b = np.asarray(got[k], np.float64), np.asarray(ref[k], np.float64)
        out[k] = float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))
    for k in PARITY_SCAL:
        out[k] = abs(float(got[k]) - float(ref[k])) / max(1.0, abs(float(ref[k])))
    out["max"] = max(out.values())
    return out


C5_FIXTURE = os.path.join(ROOT, "tests", "golden", "c5_n1_outputs.json")
FITC_VECS = ("loo_mu", "loo_var", "pred_mu", "pred_var")


def rccl_identity(ctl, glib):
    """Which RCCL every rank runs (gps_rccl_info): ncclGetVersion and the file that holds
    ncclAllReduce.  torch is imported before libgpscore in this process (the gloo control plane),
    so the library's librccl.so.1 and libamdhip64 resolve to torch's bundled copies — one HIP
    runtime per process — rather than /opt/rocm's."""
    v, path = glib.rccl_info()
    per = ctl.gather([v, path])
    return {"version": v, "version_str": "%d.%d.%d" % (v // 10000, v // 100 % 100, v % 100),
            "path": path, "all_ranks_same": all(p == per[0] for p in per),
            "why": "torch (imported first for the gloo control plane) bundles librccl.so with "
                   "SONAME librccl.so.1; the library's DT_NEEDED librccl.so.1 binds to it, as its "
                   "libamdhip64 binds to torch's bundled HIP runtime"}


def comm_check(ctl, world, rank, local, info, kind="rccl"):
    """Every rank's communicator as the library reports it (gps_comm_info: RCCL's own
    ncclCommCount / ncclCommUserRank), gathered over the control plane: the run's ranks agree
    when each communicator counts `world` ranks of the expected kind and the user ranks are a
    permutation of 0..world−1 equal to the launcher's RANKs."""
    seen = ctl.gather([rank, local] + list(info))
    agree = (all(n == world and k == kind for _, _, n, _, k in seen)
             and sorted(ur for _, _, _, ur, _ in seen) == list(range(world))
             and all(r == ur for r, _, _, ur, _ in seen))
    return {"ranks_seen": sorted({n for _, _, n, _, _ in seen}), "all_ranks_agree": bool(agree),
            "per_rank": [{"rank": r, "local_rank": lr, "comm_count": n, "comm_user_rank": ur,
                          "kind": k} for r, lr, n, ur, k in seen]}


# SURVEY.md §8e / DESIGN §8: the FITC unit's main-stream phases (gps_phase_enable) grouped by what
# scales with the ranks.  replicated: K̃mm + Lm's factorisation, B's unpack + Lb's, c = B⁻¹b;
# sharded: Knm, the q / r row norms with λ and the LOO terms, B's SYRK; exposed exchange: the main
# stream's wait for B's last chunked all-reduce and the scalar all-reduce; the rest of the unit
# (predict with its score sums) is what the unit time leaves.
SPLIT = {"replicated": ("kmm_lm", "lb", "c"), "sharded": ("knm", "q", "syrk", "r"),
         "exposed_exchange": ("exchange", "scal")}


def scaling_split(ph, steps, world, ms_unit):
    """Per-unit ms of each group of phases and the all-reduce record of one rank: B's exchange
    (the all-reduces of >= 64 KiB: its row blocks, b and the two scalars ride in the last) with
    its bytes per unit and the ring bus rate 2(N−1)/N · bytes / time (NCCL's busbw convention;
    each all-reduce timed on its own stream, so the time includes any wait for the slowest
    rank), and the small ones (score / LOO scalars)."""
    pm = {k: v["ms"] / steps for k, v in ph.get("phases", {}).items()}
    out = {"phases_ms": pm}
    for g, names in SPLIT.items():
        out[g + "_ms"] = sum(pm.get(k, 0.0) for k in names)
    out["predict_and_rest_ms"] = ms_unit - sum(pm.values()) if pm else None
    big = [(b, ms) for b, ms in ph.get("allreduce", []) if b >= 65536]
    small = [(b, ms) for b, ms in ph.get("allreduce", []) if b < 65536]
    b_bytes = sum(b for b, _ in big) / steps
    b_ms = sum(ms for _, ms in big) / steps
    out["allreduce_B"] = {"count": len(big) / steps, "bytes": b_bytes, "ms": b_ms,
                          "bus_GBps": (2.0 * (world - 1) / world * b_bytes / (b_ms * 1e-3) / 1e9)
                          if b_ms > 0 and world > 1 else None}
    out["allreduce_small"] = {"count": len(small) / steps,
                              "ms": sum(ms for _, ms in small) / steps}
    return out


# The kernel-accounting pass's FITC kernel classes that every rank repeats (the m×m work: K̃mm, the
# two factorisations with their recursion products and trailing SYRKs, B's slab sum / unpack,
# c = B⁻¹b); everything else scales with the rank's rows; allreduce_B is the exchange.
REPLICATED_TAGS = ("potrf_dag", "gemm_trmm_l", "gemm_trmm_m", "gemm_trmm_s", "gemm_syrk_m",
                   "gemm_syrk_s", "gemm_m", "gemm_s", "gram_kmm", "fitc_c", "syrk_slab_sum")


def scaling_model(prof, steps, world):
    """Per-rank kernel time (single stream, hipEvents per launch) split into replicated, sharded
    and exchange kernels, and the compute-only projection to other rank counts: replicated +
    sharded·world/N (the exchange is what the N > 1 lines measure: scaling_split.allreduce_B)."""
    ks = kernel_summary(prof, steps)
    rep_ms = sum(v["ms"] for k, v in ks.items() if k in REPLICATED_TAGS)
    ex_ms = sum(v["ms"] for k, v in ks.items() if k.startswith("allreduce"))
    sh_ms = sum(v["ms"] for k, v in ks.items()) - rep_ms - ex_ms
    return {"replicated_kernels_ms": rep_ms, "sharded_kernels_ms": sh_ms, "exchange_kernels_ms": ex_ms,
            "replicated_tags": [k for k in ks if k in REPLICATED_TAGS],
            "compute_projection_ms": {str(n): rep_ms + sh_ms * world / n for n in (1, 2, 4, 8)}}


def split_summary(splits):
    """The gathered per-rank scaling splits and their maxima over the ranks (the slowest rank sets
    the strong-scaling step)."""
    keys = [k for k, v in splits[0].items() if k.endswith("_ms") and isinstance(v, (int, float))]
    return {"per_rank": splits,
            "max_over_ranks": {k: max(sp[k] for sp in splits) for k in keys},
            "note": "main-stream phases of the production unit (events on), grouped replicated / "
                    "sharded / exposed exchange (bench.SPLIT); with m_pad > 20 tiles (C5) the row "
                    "norms' pre-pass over the top-level L11^-1 columns runs beside the recursion, "
                    "inside kmm_lm and lb (scaling_model splits by kernel instead)"}


def sample_indices(n):
    """Global row indices whose values the C5 fixture keeps: 48 evenly spaced rows plus both
    sides of every shard boundary of 2, 4 and 8 ranks (gpscore.dist.shard_rows), where an
    off-by-one in the shard bookkeeping would show."""
    from gpscore.dist import shard_rows
    idx = set(int(i) for i in np.linspace(0, n - 1, 48))
    for p in (2, 4, 8):
        for r in range(1, p):
            a, _ = shard_rows(n, p, r)
            idx.update((a - 1, a))
    return sorted(i for i in idx if 0 <= i < n)


def fitc_outputs(ctl, fgp, thf, fc, rows, test_rows):
    """The sharded C5 unit's outputs made rank-independent: the global objectives and test scores
    (every rank holds them), and for each of LOO μ/σ² (rows) and predictive μ/σ² (test rows) the
    all-rank sums Σv, Σv², Σ|v|, max|v| and the values at `sample_indices` — gathered over the gloo
    control plane, so N ranks and one rank report the same quantities (K20:222-234, 270-296)."""
    r = fgp.fit(theta=thf)
    mu, var, sc = fgp.predict(with_scores=True)
    local = {"loo_mu": (r.mu_loo, rows[0], fc["n"]), "loo_var": (r.var_loo, rows[0], fc["n"]),
             "pred_mu": (mu, test_rows[0], fc["nt"]), "pred_var": (var, test_rows[0], fc["nt"])}
    mine = {}
    for k, (v, off, n) in local.items():
        v = np.asarray(v, np.float64)
        samp = {i: float(v[i - off]) for i in sample_indices(n) if off <= i < off + len(v)}
        mine[k] = {"sum": float(v.sum()), "sumsq": float(v @ v), "sumabs": float(np.abs(v).sum()),
                   "maxabs": float(np.abs(v).max()) if len(v) else 0.0, "count": int(len(v)),
                   "samples": samp}
    everyone = ctl.gather(mine)
    vecs = {}
    for k in FITC_VECS:
        parts = [e[k] for e in everyone]
        samples = {}
        for p in parts:
            samples.update(p["samples"])
        vecs[k] = {"sum": float(sum(p["sum"] for p in parts)),
                   "sumsq": float(sum(p["sumsq"] for p in parts)),
                   "sumabs": float(sum(p["sumabs"] for p in parts)),
                   "maxabs": max(p["maxabs"] for p in parts),
                   "count": int(sum(p["count"] for p in parts)),
                   "samples": {str(i): samples[i] for i in sorted(samples)}}
    return {"objectives": dict(r.objectives), "scores": dict(sc), "vectors": vecs}


def compare_fitc_outputs(got, ref):
    """Errors of `got` against the committed N = 1 outputs `ref` (same quantities, fitc_outputs),
    each as a normwise relative error: scalars |a − b| / max(1, |b|); sampled entries
    max|a_i − b_i| / max|b|; Σv and Σ|v| relative to Σ|b|, Σv² to Σb².  The bar is the fixture's
    `tol` (50·κ·ε at C5: the C5 tests' absolute cap, κ = cond(K̃mm)(sf² + σ²)/σ²)."""
    errs = {}
    for grp in ("objectives", "scores"):
        for k, b in ref[grp].items():
            errs[f"{grp}.{k}"] = abs(float(got[grp][k]) - b) / max(1.0, abs(b))
    for k, rv in ref["vectors"].items():
        gv = got["vectors"][k]
        if gv["count"] != rv["count"] or set(gv["samples"]) != set(rv["samples"]):
            errs[f"{k}.layout"] = float("inf")
            continue
        scale = max(rv["maxabs"], 1e-300)
        errs[f"{k}.samples"] = max(abs(gv["samples"][i] - rv["samples"][i]) for i in rv["samples"]) / scale
        errs[f"{k}.sum"] = abs(gv["sum"] - rv["sum"]) / max(rv["sumabs"], 1e-300)
        errs[f"{k}.sumabs"] = abs(gv["sumabs"] - rv["sumabs"]) / max(rv["sumabs"], 1e-300)
        errs[f"{k}.sumsq"] = abs(gv["sumsq"] - rv["sumsq"]) / max(rv["sumsq"], 1e-300)
        errs[f"{k}.maxabs"] = abs(gv["maxabs"] - rv["maxabs"]) / scale
    tol = float(ref["tol"])
    worst = max(errs, key=lambda k: errs[k])
    return {"vs": f"committed N = 1 outputs ({os.path.relpath(C5_FIXTURE, ROOT)}, "
                  f"{ref.get('source', '')})",
            "tol": tol, "max_err": errs[worst], "worst": worst, "ok": bool(errs[worst] <= tol),
            "errors": errs}


def gpu_unit_outputs(gp, th, rbf=False):
    r = gp.fit(theta=th, rbf=rbf)
    mu, var, sc = gp.predict(with_scores=True)
    out = dict(r.objectives)
    out.update(loo_mu=r.mu_loo, loo_var=r.var_loo, pred_mu=mu, pred_var=var)
    out.update(sc)
    return out


def synth_c1(n=500, nt=500, seed=1):
    """C1: the SIMPLE-DATA generator (SD:158-181) at n = 500 — x = 2·N(0, 1), y ~ MVN(0,
    rbf(x, x; log k² = 0, log ℓ² = 0) + 0.3²·I), split train / test — drawn with numpy (the
    reference draws with torch.manual_seed(100 j)); the fit uses the rbf kernel at the
    generating hyper-parameters (log sf² = 0, b = log ℓ² = 0, log σ² = log 0.09)."""
    rng = np.random.default_rng(seed)
    x = 2.0 * rng.standard_normal(n + nt)
    K = np.exp(-0.5 * (x[:, None] - x[None, :]) ** 2) + 0.09 * np.eye(n + nt)
    yy = np.linalg.cholesky(K) @ rng.standard_normal(n + nt)
    th = (0.0, 0.0, np.log(0.09))
    return x[:n, None], yy[:n], x[n:, None], yy[n:], th


def c1_leg(ctx, steps):
    """BASELINE.json configs[0]: the SIMPLE-DATA full GP at n = 500, d = 1, rbf — the GPU
    unit, the torch-CPU ref-mirror of the same unit (median of 5), and their parity."""
    import gpscore
    O, RT = _oracle()
    X, y, Xt, yt, th = synth_c1()
    gp = gpscore.GP(ctx=ctx)
    gp.set_data(X, y)
    gp.set_test(Xt, yt)
    got = gpu_unit_outputs(gp, th, rbf=True)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        gp.fit(theta=th, rbf=True, return_loo=False)
        gp.predict(with_scores=True)
    ctx.synchronize()
    ms_gpu = 1e3 * (time.perf_counter() - t0) / steps
    cores = _torch_threads()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        ref = RT.ref_full(X, y, Xt, yt, *th, kind="rbf")
        ts.append(time.perf_counter() - t0)
    return {"config": "C1 SIMPLE-DATA full GP n=500 d=1 rbf, n*=500 (SD:158-213 generator)",
            "ms_per_step": ms_gpu, "cpu_ref_ms": 1e3 * float(np.median(ts)), "cpu_cores": cores,
            "speedup_vs_cpu": float(np.median(ts)) * 1e3 / ms_gpu, "parity": parity(got, ref),
            "note": "host round trips included: at n = 500 the unit is launch/PCIe bound"}


def surface_leg(ctx, steps, with_cpu):
    """contour-plot.R's four objective surfaces (CP.R:43-85) on its 50 × 50
    (length-scale, noise s.d.) grid at n = 20 (CP.R:88-141): 2500 small full GPs, one wavefront
    each, per call.  CPU: the oracle's numpy ref-mirror of the same grid (CP.R's op sequence)."""
    import gpscore
    O, _ = _oracle()
    x, y = O.cp_data(seed=0)
    ell, sd = np.linspace(0.01, 2.0, 50), np.linspace(0.01, 1.0, 50)
    got = gpscore.surface(x, y, ell, sd, ctx=ctx)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        gpscore.surface(x, y, ell, sd, ctx=ctx)
    ms = 1e3 * (time.perf_counter() - t0) / steps
    res = {"config": "CP.R grid 50 x 50 (l in [0.01, 2], noise s.d. in [0.01, 1]), n = 20, d = 1",
           "ms_per_surface": ms, "grid_points_per_s": 2500 / (ms * 1e-3),
           "note": "4 objectives per grid point (LOO-CRPS, in-sample CRPS, NLML, LOO-LogS); host "
                   "round trip included"}
    if with_cpu:
        t0 = time.perf_counter()
        ref = O.cp_surface(x, y, ell, sd)
        res["cpu_ref_ms"] = 1e3 * (time.perf_counter() - t0)
        res["parity_max_nrel"] = max(
            float(np.max(np.abs(got[k] - ref[i])) / np.max(np.abs(ref[i])))
            for i, k in enumerate(("loo_crps", "insample_crps", "nlml", "loo_logs")))
    return res


def fitc_cpu_baseline():
    """FITC at C4 on the host (BASELINE.md:56-57): the dense torch ref-mirror (K20:222-234,
    329-340, 434-447, 270-296: n×n big_Q, chol_solve = potrf + 2 LU) timed at
    (n, n*) = (5000, 1250) and (10000, 2500) with C4's m = 2000 and d = 8, extrapolated
    as n³ (n* ∝ n) to (40000, 10000) — a 12.8 GB n×n matrix per copy, ~20 min — and the
    O(n·m²) Woodbury numpy restatement timed directly at C4."""
    O, RT = _oracle()
    cores = _torch_threads()
    c = CONFIGS["C4"]
    times = {}
    for n in (5000, 10000):
        X, y, Xt, yt, Z, th = synth(n, c["d"], n // 4, c["seed"], c["m"])
        t0 = time.perf_counter()
        RT.ref_fitc(X, y, Xt, yt, Z, *th)
        times[n] = time.perf_counter() - t0
    extrap = times[10000] * (c["n"] / 10000) ** 3
    X, y, Xt, yt, Z, th = synth(c["n"], c["d"], c["nt"], c["seed"], c["m"])
    t0 = time.perf_counter()
    O.fast_fitc(X, y, Xt, yt, Z, *th)
    t_fast = time.perf_counter() - t0
    return {"value": 1.0 / extrap, "unit": "fit+predict+score units/s (C4)", "cores": cores,
            "kind": "port",
            "sample": f"dense torch-CPU ref-mirror FITC at n=5000 / 10000 (n*=n/4, m=2000, d=8): "
                      f"{times[5000]:.1f} / {times[10000]:.1f} s, n^3-extrapolated to C4: "
                      f"{extrap:.0f} s per unit",
            "woodbury_numpy_s": t_fast,
            "woodbury_note": "O(n·m²) numpy/LAPACK restatement (the GPU's algorithm) on the full C4 "
                             "unit — not the reference algorithm"}


def c5_tol(Z, th):
    """50·κ·ε, κ = cond(K̃mm)(sf² + σ²)/σ² from the host eigenvalues of the jittered K(Z, Z):
    the absolute cap the C5 parity tests hold every output to (tests/test_gpu_parity.py
    fitc_cap), stored with the fixture."""
    O, _ = _oracle()
    Kmm = O.fast_gram(Z, Z, th[0], th[1], diag_add=O.FITC_JITTER)
    ev = np.linalg.eigvalsh(Kmm)
    sf2, sn2 = np.exp(th[0]), np.exp(th[2])
    return float(50.0 * (ev[-1] / ev[0]) * (sf2 + sn2) / sn2 * np.finfo(np.float64).eps)


def host_gpu():
    try:
        import torch
        return torch.cuda.get_device_properties(0).name or "MI355X"
    except Exception:  # noqa: BLE001
        return "one MI355X"


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout): a long run keeps writing, so a
    watchdog that reads silence as a hang sees the legs go by."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-fitc", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-grad", action="store_true")
    ap.add_argument("--no-block", action="store_true", help="skip the block-LOO (next-2) leg")
    ap.add_argument("--no-tiny-gemm", action="store_true",
                    help="64-tile split-K path for the small GEMMs instead of the 16x16-per-wave kernel")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--fitc-traffic-json", default=os.path.join(ROOT, "profiles", "fitc_traffic.json"))
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 control-plane rehearsal on a 1-GPU box: every rank on device 0, "
                         "no RCCL communicator (FITC objectives then cover the local shard only)")
    ap.add_argument("--one-gpu-rccl", action="store_true",
                    help="functional test of the N>1 RCCL path on a 1-GPU box: every rank on device 0 "
                         "with a REAL RCCL communicator — each rank presents its own NCCL_HOSTID, so "
                         "RCCL's one-rank-per-GPU check passes and the ranks exchange over loopback "
                         "sockets; the rank-count and C5-vs-N=1 checks run as at N>1 (not a "
                         "performance run: the ranks share one GPU)")
    ap.add_argument("--write-c5-fixture", metavar="PATH", default=None,
                    help="N = 1 only: write the C5 unit's rank-independent outputs (fitc_outputs) "
                         "to PATH — the fixture tests/golden/c5_n1_outputs.json that N > 1 runs "
                         "are checked against")
    ap.add_argument("--dry", action="store_true",
                    help="launcher / control-plane check: ranks meet over gloo, agree on the world "
                         "size and print the JSON skeleton without touching the GPU")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    # --gpus N with no launcher around us: this process becomes the spawner, before any GPU call
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, args.one_gpu_rccl))
    world, rank, local = dist_env()
    if world != args.gpus:
        print(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a "
              f"{world}-process run as {args.gpus} GPUs", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.dry and os.environ.get("GPS_BENCH_DRY_FAIL") == str(rank):
        sys.exit(3)  # launcher test: one rank dies before the control plane forms
    ctl = Ctl(world)
    if args.dry:
        # every rank reports its (rank, local rank) over the control plane; rank 0 checks the set
        me = [rank, local, os.getpid()]
        everyone = [me]
        if ctl.dist:
            everyone = [None] * world
            ctl.dist.all_gather_object(everyone, me)
        if os.environ.get("GPS_BENCH_DRY_SLEEP"):  # launcher test: ranks that are still running
            time.sleep(float(os.environ["GPS_BENCH_DRY_SLEEP"]))
        # the rank-count check of the FITC leg, on a stand-in for gps_comm_info (no GPU here);
        # GPS_BENCH_DRY_COMM_COUNT makes one rank's stand-in report a wrong count
        bad = os.environ.get("GPS_BENCH_DRY_COMM_COUNT", "")
        n_seen = int(bad.split(":")[1]) if bad and bad.split(":")[0] == str(rank) else world
        rc = comm_check(ctl, world, rank, local, (n_seen, rank, "dry"), kind="dry")
        from gpscore import _lib as glib  # (loads the library; gps_rccl_info needs no device)
        rc["library"] = rccl_identity(ctl, glib)
        # the N > 1 scaling split on a stand-in phase record (no GPU): the same code and schema
        stand_in = {"phases": {k: {"count": 1, "ms": 1.0} for g in SPLIT.values() for k in g},
                    "allreduce": [[8.0 * 4000 * 4001 / 2 / 4, 1.0]] * 4 + [[16.0, 0.05]]}
        split = scaling_split(stand_in, 1, world, 20.0)
        if rank == 0:
            ok = sorted(r for r, _, _ in everyone) == list(range(world)) and \
                len({p for _, _, p in everyone}) == world
            line = {"metric": METRIC, "value": None, "n_gpus": world, "dry": True,
                    "ranks": everyone, "ranks_ok": ok, "steps": args.steps,
                    "warmup": args.warmup,
                    "fitc": {"rccl": rc, "C5": {"scaling_split": split_summary([split] * world)}}}
            if not rc["all_ranks_agree"]:
                line["failures"] = [f"communicators disagree with --gpus {world}"]
            print(json.dumps(line))
        if ctl.dist:
            ctl.dist.destroy_process_group()
        if not rc["all_ranks_agree"]:
            sys.exit(4)
        return
    import gpscore
    failures = []  # self-checks that fail the run (non-zero exit) after the JSON line
    ctx = gpscore.Context(0 if (args.rehearse or args.one_gpu_rccl) else local)
    if args.no_tiny_gemm:
        ctx.set_tiny_gemm(False)
    gp = gpscore.GP(ctx=ctx)

    # ---------------- full GP (replicas) ----------------
    c = CONFIGS[args.config]
    X, y, Xt, yt, _, th = synth(c["n"], c["d"], c["nt"], c["seed"])
    gp.set_data(X, y)
    gp.set_test(Xt, yt)

    def unit():
        gp.fit(theta=th, return_loo=False)
        return gp.predict(with_scores=True)

    log(f"{args.config}: warmup")
    for _ in range(args.warmup):
        unit()
    log(f"{args.config}: timed pass")
    # headline pass: production configuration (side-stream overlap on, no events)
    t_full = timed(ctl, ctx, unit, args.steps)
    ms_full = 1e3 * t_full / args.steps
    # kernel-accounting pass: same steps, one stream, hipEvents around every launch
    prof, ms_acct = kernel_pass(ctl, ctx, unit, args.steps)
    def upload():
        gp.set_data(X, y)
        gp.set_test(Xt, yt)
    unit_phases = phases(ctl, ctx, gp, th, args.steps, prof, ms_full, upload)
    got = gpu_unit_outputs(gp, th)  # every output of the unit, for the parity record
    obj = {k: got[k] for k in ("nlml", "loo_crps", "loo_logs", "logdet", "quad")}
    sc = {k: got[k] for k in ("test_crps", "test_logs", "test_msll", "test_smse", "test_mse",
                              "test_cover")}

    # HBM bytes per launch from the committed rocprofv3 counter passes
    # (tools/profile_round.sh -> tools/traffic.py; counters cannot be read live here)
    def read_traffic(path):
        try:
            tr = json.load(open(path)).get("_roofline", {})
            return tr.get("gemm_per_launch_bytes"), tr.get("gram_per_launch_bytes")
        except Exception:  # noqa: BLE001 - absent / unreadable file: traffic stays null
            return None, None
    traffic, traffic_gram = read_traffic(args.traffic_json)

    res = {
        "metric": METRIC,
        "value": world * args.steps / t_full,
        "unit": f"fit+predict+score units/s ({args.config} full GP, whole job)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_full,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic (SURVEY.md §8d generator; random-init theta fixed)",
        "config": {"workload": f"{args.config} full GP fit(NLML+LOO-CRPS+LOO-LogS)+predict+score",
                   "n": c["n"], "d": c["d"], "n_test": c["nt"], "kernel": "ARD",
                   "parallelism": (("replicas on ONE GPU, RCCL functional test (--one-gpu-rccl)"
                                    if args.one_gpu_rccl else "replicas") if world > 1 else "single")},
        "roofline": roofline_mfma(prof, traffic, args.steps, alg_flop("full", c)),
        "roofline_gram": roofline_gram(prof, args.steps, traffic_gram),
        "roofline_trailing_update": roofline_trailing(prof, args.steps),
        "objectives": obj, "scores": sc,
        "kernels_per_step": kernel_summary(prof, args.steps),
        "phases": unit_phases,
        "kernel_accounting": {"ms_per_step": ms_acct, "streams": 1,
                              "note": "second timed pass, overlap off, hipEvents around each launch"},
    }

    log("headline done: %.2f ms/step" % ms_full)
    # ---------------- gradients (next-1: one GD iteration = fwd + analytic bwd) -------------
    if not args.no_grad:
        grad = {}
        n_pad = -(-c["n"] // 128) * 128
        for objective, flop in (("nlml", n_pad ** 3 * 1.0), ("loo_crps", n_pad ** 3 * 2.0)):
            def gstep():
                return gp.value_and_grad(th, objective)
            gstep()
            tg = timed(ctl, ctx, gstep, max(1, args.steps // 2))
            ms = 1e3 * tg / max(1, args.steps // 2)
            grad[objective] = {"ms_per_iteration": ms, "flop": flop,
                               "tflops": flop / (ms * 1e-3) / 1e12}
        res["grad"] = {"config": args.config, "note": "value_and_grad per GD iteration "
                       "(fit + A^-1 + [A^-1 diag(c) A^-1] + dA/dtheta contraction); flop = n^3 "
                       "(NLML) / 2n^3 (LOO) at n_pad", **grad}

    log("gradient leg done")
    # ---------------- next-2: block-LOO objectives, one GD iteration each (C2) ----------------
    if not args.no_block:
        from gpscore.gp import es_draws
        cb = CONFIGS["C2"]
        Xb, yb, _, _, _, thb = synth(cb["n"], cb["d"], cb["nt"], cb["seed"])
        bgp = gpscore.GP(ctx=ctx)
        bgp.set_data(Xb, yb)
        draws = es_draws(cb["n"], 4, 300, np.random.default_rng(0))
        blk = {}
        for objective in ("dss", "kc", "es"):
            kw = {"num_sim": 300, "draws": draws} if objective == "es" else {}

            def bstep():
                return bgp.block_loo(thb, objective, grad=True, **kw)
            bstep()
            k = max(1, args.steps // 2)
            blk[objective] = {"ms_per_iteration": 1e3 * timed(ctl, ctx, bstep, k) / k}
        res["block_loo"] = {"config": f"C2 full GP n={cb['n']}, 4 folds of {cb['n'] // 4}; ES with "
                            "300 draws per fold (KF:652-655)",
                            "note": "value + analytic gradient per GD iteration (KF:487-543, "
                                    "K20:655-720, KF:607-663)", **blk}

    log("block-LOO leg done")
    # ---------------- FITC (rows sharded, RCCL all-reduce) ----------------
    if not args.no_fitc:
        from gpscore.dist import shard_rows
        fitc = {}
        legs = ["C5"] + (["C4"] if world == 1 else [])
        fgp = gpscore.GP(ctx=ctx)
        comm_err = None
        if world > 1 and not args.rehearse:
            import ctypes
            lib = gpscore.load()
            uid = None
            if rank == 0:
                buf = ctypes.create_string_buffer(128)
                ctx.check(lib.gps_comm_unique_id(buf), "gps_comm_unique_id")
                uid = buf.raw
            obj_l = [uid]
            ctl.dist.broadcast_object_list(obj_l, src=0)
            info = None
            try:
                ctx.call("gps_comm_init", world, rank, ctypes.create_string_buffer(obj_l[0], 128))
                info = ctx.comm_info()
            except Exception as e:  # noqa: BLE001 - reported in the JSON line, not fatal
                comm_err = repr(e)
            # every rank learns whether any communicator failed (over gloo, so no rank is
            # left waiting in an RCCL collective); the headline is already measured
            if ctl.max(1.0 if comm_err else 0.0) > 0:
                legs = []
                fitc["error"] = comm_err or "gps_comm_init failed on another rank"
            else:
                fitc["rccl"] = comm_check(ctl, world, rank, local, info)
                fitc["rccl"]["library"] = rccl_identity(ctl, gpscore._lib)
                if not fitc["rccl"]["all_ranks_agree"]:
                    failures.append(f"RCCL communicators disagree with --gpus {world}: "
                                    f"{fitc['rccl']['per_rank']}")
                    legs = []
        for leg in legs:
            fc = CONFIGS[leg]
            Xf, yf, Xtf, ytf, Z, thf = synth(fc["n"], fc["d"], fc["nt"], fc["seed"], fc["m"])
            a, b = shard_rows(fc["n"], world, rank)
            ta, tb = shard_rows(fc["nt"], world, rank)
            fgp.set_data(Xf[a:b], yf[a:b], kind="fitc", Z=Z, n_total=fc["n"],
                         ytr_stats=(float(yf.mean()), float(yf.var(ddof=1))))
            fgp.set_test(Xtf[ta:tb], ytf[ta:tb], nt_total=fc["nt"])

            def funit():
                fgp.fit(theta=thf, return_loo=False)
                return fgp.predict(with_scores=True)

            log(f"FITC {leg}: warmup")
            for _ in range(args.warmup):
                funit()
            tf = timed(ctl, ctx, funit, args.steps)
            # the same production schedule with phase events (after the headline pass: the
            # events are not in `value`), every rank's split gathered
            ctx.phases(True)
            tph = timed(ctl, ctx, funit, args.steps)
            ctx.phases(False)
            split = scaling_split(ctx.phase_collect(), args.steps, world, 1e3 * tph / args.steps)
            split["unit_ms_with_events"] = 1e3 * tph / args.steps
            splits = ctl.gather(split)
            fprof, fms_acct = kernel_pass(ctl, ctx, funit, args.steps)
            fphases = phases(ctl, ctx, fgp, thf, args.steps, fprof, 1e3 * tf / args.steps)
            fobj = fgp.fit(theta=thf, return_loo=False).objectives
            fout = None
            if leg == "C5" and not args.rehearse:  # outside the timed passes
                fout = fitc_outputs(ctl, fgp, thf, fc, (a, b), (ta, tb))
            fitc[leg] = {"ms_per_step": 1e3 * tf / args.steps,
                         "units_per_s": args.steps / tf,
                         "config": {"n": fc["n"], "m": fc["m"], "d": fc["d"], "n_test": fc["nt"],
                                    "rows_per_rank": b - a, "ranks": world},
                         "scaling": "strong",
                         "objectives": fobj,
                         "roofline": roofline_mfma(
                             fprof, read_traffic(args.fitc_traffic_json)[0] if leg == "C4" else None,
                             args.steps, alg_flop("fitc", fc, world)),
                         "kernel_accounting_ms_per_step": fms_acct,
                         "phases": fphases,
                         "scaling_split": split_summary(splits),
                         "scaling_model": scaling_model(fprof, args.steps, world),
                         "kernels_per_step": kernel_summary(fprof, args.steps)}
            if fout is not None:
                if args.write_c5_fixture and world == 1 and rank == 0:
                    fixture = dict(fout, config=dict(fc), theta=[thf[0], list(thf[1]), thf[2]],
                                   tol=c5_tol(Z, thf), source=f"bench.py N = 1 on {host_gpu()}")
                    with open(args.write_c5_fixture, "w") as f:
                        json.dump(fixture, f, indent=1, sort_keys=True)
                    log(f"C5 fixture written to {args.write_c5_fixture}")
                if os.path.exists(C5_FIXTURE):
                    with open(C5_FIXTURE) as f:
                        cmp = compare_fitc_outputs(fout, json.load(f))
                    fitc[leg]["parity_vs_n1"] = cmp
                    if not cmp["ok"]:
                        failures.append(f"C5 at N = {world} differs from the N = 1 fixture: "
                                        f"{cmp['worst']} {cmp['max_err']:.3g} > {cmp['tol']:.3g}")
                else:
                    fitc[leg]["parity_vs_n1"] = {"error": f"{C5_FIXTURE} missing"}
                    if world > 1:
                        failures.append("no N = 1 fixture to check the sharded C5 unit against")
            if not args.no_grad:  # next-1: one FITC GD iteration (theta and Z), K20:222-247
                fg = {}
                for objective in ("nlml", "loo_crps"):
                    def fgstep():
                        return fgp.value_and_grad(thf, objective)
                    fgstep()
                    k = max(1, args.steps // 2)
                    fg[objective] = {"ms_per_iteration": 1e3 * timed(ctl, ctx, fgstep, k) / k}
                if leg == "C4" and world == 1 and not args.no_block:  # next-2: K20:655-726 KC,
                    for bobj in ("kc", "dss"):                        # K20:523-587 DSS
                        def fbstep():
                            return fgp.block_loo(thf, bobj, grad=True)
                        fbstep()
                        fg["block_" + bobj] = {"ms_per_iteration": 1e3 * timed(ctl, ctx, fbstep, 1),
                                               "note": "4 folds of 10 000 rows, theta and Z gradient "
                                                       "(folds in low rank, DESIGN.md §10)"}
                fitc[leg]["grad"] = fg
            del Xf, yf, Xtf, ytf
        if world > 1 and not args.rehearse and "error" not in fitc:
            ctx.call("gps_comm_destroy")
        res["fitc"] = fitc

    log("FITC legs done")
    res["surface"] = surface_leg(ctx, args.steps, rank == 0 and world == 1 and not args.no_cpu)
    if rank == 0 and world == 1 and not args.no_cpu:
        log("CPU baseline (about two minutes)")
        cb, ref = cpu_baseline(args.config)
        res["cpu_baseline"] = cb
        res["speedup_vs_cpu"] = res["value"] / cb["value"]
        res["parity"] = {"vs": f"torch-CPU ref-mirror (reference op sequence) on the same "
                               f"{args.config} inputs",
                         "metric": "normwise relative error (vectors: max|a-b|/max|b|; scalars: "
                                   "|a-b|/max(1,|b|))", **parity(got, ref)}
        log("C1 leg")
        res["c1"] = c1_leg(ctx, args.steps)
        if "fitc" in res and "C4" in res["fitc"]:
            log("FITC C4 CPU baseline")
            res["fitc"]["C4"]["cpu_baseline"] = fitc_cpu_baseline()
    if args.rehearse:
        res["rehearsal"] = "all ranks on device 0, no RCCL: not a measurement"
    if failures:
        res["failures"] = failures
    if rank == 0:
        print(json.dumps(res))
    if ctl.dist:
        ctl.dist.destroy_process_group()
    if failures:  # the line is printed (it carries the evidence), but the run fails
        for f in failures:
            print(f"[bench] FAILED: {f}", file=sys.stderr, flush=True)
        sys.exit(4)


if __name__ == "__main__":
    main()
