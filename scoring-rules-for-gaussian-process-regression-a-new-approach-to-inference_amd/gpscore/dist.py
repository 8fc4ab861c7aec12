"""Multi-GPU FITC: one process per GPU, rows of Knm sharded, one RCCL all-reduce.

SURVEY.md §8e: every rank holds a contiguous slice of the training rows (and of
the test rows), replicates the m×m factors, and contributes its additive
partials {B_p = Kmn_pΛ_p⁻¹Knm_p, b_p, Σlogλ, Σy²/λ} to ONE in-library
``ncclAllReduce`` (sum, fp64) per objective evaluation; the LOO / test score
sums are all-reduced as 2 / 6 scalars.  The communicator is created inside
libgpscore.so (RCCL over xGMI); torch.distributed (any backend) is only used
to broadcast the 128-byte unique id and the global target statistics.

The full GP does not shard (a distributed Cholesky is out of scope): under
``torchrun`` it runs as independent replicas, one per GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def shard_rows(n, nranks, rank):
    """Contiguous split of n rows over nranks; the first n % nranks ranks get one
    extra row.  Returns (start, stop)."""
    if not 0 <= rank < nranks:
        raise ValueError("rank out of range")
    q, r = divmod(int(n), int(nranks))
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def fold_shard_rows(n, nfold, nranks, rank):
    """Rows of `rank` when n rows in nfold block-LOO folds ([int(f·n/k), int((f+1)·n/k)),
    KF:496-499) are sharded over nranks on fold boundaries: the folds are split as evenly as
    shard_rows splits rows, so every fold lies inside one rank's rows — what the sharded
    FITC block-LOO (gps_fitc_blockloo) needs.  Returns (start, stop)."""
    if not 1 <= nranks <= nfold:
        raise ValueError("need 1 <= nranks <= nfold (every rank holds at least one fold)")
    f0, f1 = shard_rows(nfold, nranks, rank)
    bound = (lambda f: int(n) if f == nfold else int(f * int(n) / nfold))
    return bound(f0), bound(f1)


def global_target_stats(y_local, group=None):
    """(mean, unbiased var, n_total) of the training targets over all ranks —
    what trivial_loss / SMSE need (KF:112-114, 130).  Two passes over float64 host
    all-reduces (works with gloo or nccl groups): [Σy, n] gives the global mean, then
    Σ(y − mean)² — no cancellation when the mean is large against the spread."""
    import torch
    import torch.distributed as dist
    y = np.asarray(y_local, dtype=np.float64).ravel()
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([y.sum(), float(y.size)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, group=group)
    s, n = (float(v) for v in t.cpu())
    mean = s / n
    c = torch.tensor([float(((y - mean) ** 2).sum())], dtype=torch.float64, device=dev)
    dist.all_reduce(c, group=group)
    var = float(c.cpu()[0]) / (n - 1) if n > 1 else 1.0
    return mean, var, int(round(n))


def broadcast_unique_id(uid_or_none, group=None, src=0):
    """Broadcast RCCL's 128-byte unique id from ``src`` (torch.distributed object
    broadcast: works on gloo and nccl)."""
    import torch.distributed as dist
    obj = [uid_or_none]
    dist.broadcast_object_list(obj, src=src, group=group)
    return obj[0]


def attach_comm(gp, group=None):
    """Create the in-library RCCL communicator for ``gp.ctx`` across the ranks of
    ``group`` (one rank per GPU)."""
    import torch.distributed as dist
    lib = _lib.load()
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    uid = None
    if rank == 0:
        buf = ctypes.create_string_buffer(128)
        rc = lib.gps_comm_unique_id(buf)
        if rc != 0:
            raise _lib.GpsError(f"gps_comm_unique_id failed: {lib.gps_last_error(None).decode()}")
        uid = buf.raw
    uid = broadcast_unique_id(uid, group)
    gp.ctx.call("gps_comm_init", world, rank, ctypes.create_string_buffer(uid, 128))
    gp.comm = (world, rank)
    return gp


class ShardedFITC:
    """FITC over this rank's row shard with the all-reduce inside libgpscore.

    ``fit`` / ``predict`` return GLOBAL objectives and scores (identical on every
    rank) and this rank's LOO / predictive vectors."""

    def __init__(self, gp, group=None):
        import torch.distributed as dist
        self.gp, self.group = gp, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        if gp.comm is None and self.world > 1:
            attach_comm(gp, group)

    def set_data(self, X_full, y_full, Z, Xt_full=None, yt_full=None):
        n = len(y_full)
        if n < self.world:
            # every rank sees the same n, so every rank raises here — none is left inside
            # an all-reduce waiting for a rank whose empty shard the library rejected
            raise ValueError(f"{n} training rows cannot be sharded over {self.world} ranks "
                             "(every rank needs at least one row)")
        a, b = shard_rows(n, self.world, self.rank)
        ytr_mean = float(np.mean(y_full))
        ytr_var = float(np.var(y_full, ddof=1))
        self.rows = (a, b)
        self.gp.set_data(X_full[a:b], y_full[a:b], kind="fitc", Z=Z, n_total=n,
                         ytr_stats=(ytr_mean, ytr_var))
        if Xt_full is not None:
            nt = len(Xt_full)
            ta, tb = shard_rows(nt, self.world, self.rank)
            self.test_rows = (ta, tb)
            self.gp.set_test(Xt_full[ta:tb], None if yt_full is None else yt_full[ta:tb],
                             nt_total=nt)
        return self

    def fit(self, theta):
        return self.gp.fit(theta=theta)

    def predict(self, with_scores=True):
        return self.gp.predict(with_scores=with_scores)
