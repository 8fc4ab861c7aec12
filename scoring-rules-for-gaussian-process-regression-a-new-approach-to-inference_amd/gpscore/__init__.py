"""gpscore — MI355X (gfx950) GP-regression hot path: Gram build, Cholesky /
log-determinant / solves, LOO and test-set CRPS / log-score, for the full GP and
the FITC sparse GP (Woodbury form, rows sharded over GPUs with RCCL).

Drop-in layers:
  * ``gpscore.compat``  — the reference scripts' helper functions, same names;
  * ``gpscore.GP``      — fit / predict / score on numpy arrays;
  * ``gpscore.dist``    — one process per GPU, FITC row sharding;
  * ``gpscore._lib``    — the ctypes binding of libgpscore.so (include/gpscore.h).
"""
from ._lib import (Context, GpsError, NotPositiveDefinite, build_id, check_build_id,  # noqa: F401
                   default_context, load, OBJ_NAMES, SCORE_NAMES)
from .gp import GP, FitResult, fit, pack_theta, score, surface  # noqa: F401

__version__ = "0.1.0"
