"""ctypes binding of libgpscore.so (C-ABI declared in include/gpscore.h).

This is the reference-side binding a maintainer adds under the reference
scripts: plain pointers and sizes, no torch types.  There is no
CPU fallback anywhere in this package: if the library is missing or no HIP
device is present, loading / context creation raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPSCORE_LIB", os.path.join(_HERE, "libgpscore.so"))
ABI_VERSION = 600  # include/gpscore.h GPS_ABI_VERSION: the signatures below are this version's
GPS_N_STATS = 6
GPS_COMM_NONE, GPS_COMM_RCCL, GPS_COMM_LOCAL = 0, 1, 2
COMM_KINDS = {GPS_COMM_NONE: "none", GPS_COMM_RCCL: "rccl", GPS_COMM_LOCAL: "local"}

GPS_ARD, GPS_RBF = 0, 1
GPS_FULL, GPS_LOWER = 0, 1
GPS_OPT_OVERLAP, GPS_OPT_GEMM_MAP, GPS_OPT_TINY_GEMM, GPS_OPT_GRAM_REG = 0, 3, 7, 9
GPS_OPT_GRAPH = 10
GPS_OPT_PRED_PRE = 11
GPS_OPT_DAG = 12
GPS_OPT_DAG_TILES = 13
GPS_OPT_DAG_GROUP = 17
GPS_OPT_STREAM_K = 18
GPS_OPT_DAG_WGS = 19
GPS_OPT_DAG_ORDER = 25
GPS_OPT_SLAB_XCD = 26
GPS_OPT_FITC_DEP = 27
GPS_OPT_AR_CHUNKS = 15
OBJ_NAMES = ("nlml", "loo_crps", "loo_logs", "logdet", "quad")
SURFACE_NAMES = ("loo_crps", "insample_crps", "nlml", "loo_logs")
GPS_SURF_LOGS_ADD_NOISE = 1
SCORE_NAMES = ("test_crps", "test_logs", "test_msll", "test_smse", "test_mse", "test_cover")

_c_int, _c_i64, _c_dbl, _c_vp, _c_cp = (ctypes.c_int, ctypes.c_int64, ctypes.c_double,
                                        ctypes.c_void_p, ctypes.c_char_p)
_P = ctypes.POINTER(ctypes.c_double)

# name -> (restype, argtypes); every symbol include/gpscore.h declares
SIGNATURES = {
    "gps_version": (_c_int, []),
    "gps_build_id": (_c_int, [_c_cp, _c_int]),
    "gps_ctx_create": (_c_int, [_c_int, ctypes.POINTER(_c_vp)]),
    "gps_ctx_destroy": (_c_int, [_c_vp]),
    "gps_last_error": (_c_cp, [_c_vp]),
    "gps_ctx_set_stream": (_c_int, [_c_vp, _c_vp]),
    "gps_ctx_stream": (_c_vp, [_c_vp]),
    "gps_ctx_synchronize": (_c_int, [_c_vp]),
    "gps_ctx_set_option": (_c_int, [_c_vp, _c_int, _c_int]),
    "gps_ctx_stats": (_c_int, [_c_vp, _c_vp, _c_int]),
    "gps_dag_task_list": (_c_int, [_c_int, _c_int, _c_vp, _c_int]),
    "gps_prof_enable": (_c_int, [_c_vp, _c_int]),
    "gps_prof_collect": (_c_int, [_c_vp, _c_cp, _c_i64]),
    "gps_phase_enable": (_c_int, [_c_vp, _c_int]),
    "gps_phase_collect": (_c_int, [_c_vp, _c_cp, _c_i64]),
    "gps_rccl_info": (_c_int, [ctypes.POINTER(_c_int), _c_cp, _c_int]),
    "gps_gram": (_c_int, [_c_vp, _c_int, _P, _c_i64, _P, _c_i64, _c_int, _c_dbl, _P, _c_int,
                          _c_dbl, _c_int, _P]),
    "gps_potrf": (_c_int, [_c_vp, _c_i64, _P, _c_i64, _P]),
    "gps_potrs": (_c_int, [_c_vp, _c_i64, _c_i64, _P, _c_i64, _P, _c_i64, _P, _c_i64]),
    "gps_diag_inv": (_c_int, [_c_vp, _c_i64, _P, _c_i64, _P]),
    "gps_gemm": (_c_int, [_c_vp, _c_int, _c_int, _c_i64, _c_i64, _c_i64, _c_dbl, _P, _c_i64, _P,
                          _c_i64, _c_dbl, _P, _c_i64]),
    "gps_scores": (_c_int, [_c_vp, _P, _P, _P, _c_i64, _c_dbl, _c_dbl, _P]),
    "gps_full_set_data": (_c_int, [_c_vp, _P, _P, _c_i64, _c_int]),
    "gps_full_set_test": (_c_int, [_c_vp, _P, _P, _c_i64]),
    "gps_full_fit": (_c_int, [_c_vp, _c_int, _P, _c_int, _P, _P, _P]),
    "gps_full_grad": (_c_int, [_c_vp, _c_int, _P, _c_int, _c_int, _P, _P]),
    "gps_full_predict": (_c_int, [_c_vp, _P, _P, _P]),
    "gps_fitc_set_data": (_c_int, [_c_vp, _P, _P, _c_i64, _c_int, _c_dbl, _c_dbl, _c_i64]),
    "gps_fitc_set_test": (_c_int, [_c_vp, _P, _P, _c_i64, _c_i64]),
    "gps_fitc_set_inducing": (_c_int, [_c_vp, _P, _c_i64]),
    "gps_fitc_fit": (_c_int, [_c_vp, _P, _c_int, _P, _P, _P]),
    "gps_fitc_grad": (_c_int, [_c_vp, _P, _c_int, _c_int, _P, _P, _P]),
    "gps_full_blockloo": (_c_int, [_c_vp, _c_int, _P, _c_int, _c_int, _c_int, _P, _P, _P]),
    "gps_full_blockloo_es": (_c_int, [_c_vp, _c_int, _P, _c_int, _c_int, _c_int, _c_dbl, _P, _P,
                                      _P, _P]),
    "gps_fitc_blockloo": (_c_int, [_c_vp, _P, _c_int, _c_int, _c_int, _P, _P, _P, _P]),
    "gps_energy_score": (_c_int, [_c_vp, _P, _P, _c_i64, _P, _c_int, _c_dbl, _P, _P]),
    "gps_fitc_predict": (_c_int, [_c_vp, _P, _P, _P]),
    "gps_fitc_intermediates": (_c_int, [_c_vp, _P, _P, _P, _P, _P]),
    "gps_full_surface": (_c_int, [_c_vp, _P, _P, _c_i64, _c_int, _c_dbl, _P, _c_i64, _P, _c_i64,
                                  _c_int, _P]),
    "gps_comm_unique_id": (_c_int, [_c_cp]),
    "gps_comm_init": (_c_int, [_c_vp, _c_int, _c_int, _c_cp]),
    "gps_comm_init_local": (_c_int, [_c_vp, _c_int, _c_int, ctypes.c_longlong]),
    "gps_comm_info": (_c_int, [_c_vp, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int),
                               ctypes.POINTER(_c_int)]),
    "gps_comm_destroy": (_c_int, [_c_vp]),
}

_lib = None


class GpsError(RuntimeError):
    """A HIP / RCCL / argument error reported by libgpscore (status < 0)."""


class NotPositiveDefinite(GpsError):
    """Cholesky hit a non-positive pivot (status > 0), as torch.potrf raises
    RuntimeError (the reference catches it at KF:726 / K20:784)."""

    def __init__(self, info, msg):
        super().__init__(msg)
        self.info = info


def load():
    """Load libgpscore.so once; raise if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libgpscore.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (or make -C <pkg>/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    lib.gps_version.restype = _c_int
    lib.gps_version.argtypes = []
    if lib.gps_version() != ABI_VERSION:  # an old library under new signatures would misread
        raise ImportError(f"{LIB_PATH} has ABI version {lib.gps_version()}, this binding "
                          f"expects {ABI_VERSION}: rebuild the library")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def rccl_info():
    """(ncclGetVersion, the file that holds ncclAllReduce as this process resolved it)."""
    lib = load()
    v = _c_int()
    buf = ctypes.create_string_buffer(4096)
    rc = lib.gps_rccl_info(ctypes.byref(v), buf, len(buf))
    if rc != 0:
        raise GpsError(f"gps_rccl_info failed ({rc})")
    return v.value, buf.value.decode()


def build_id():
    """The source hash the loaded library was built from (gps_build_id)."""
    lib = load()
    buf = ctypes.create_string_buffer(80)
    lib.gps_build_id(buf, len(buf))
    return buf.value.decode()


def check_build_id():
    """Refuse a library that was not built from the sources checked out beside it: the test
    suite and smoke() call this, so a passing GPU record names the HEAD sources' build.  Returns
    the id; when the sources are absent (a deployed library) nothing is compared."""
    from . import buildid
    want = buildid.source_hash()
    got = build_id()
    if want is not None and got != want:
        raise ImportError(f"{LIB_PATH} was built from other sources (build id {got[:16]}, the "
                          f"checked-out csrc/ hashes to {want[:16]}): rebuild it with "
                          "`make -C <pkg>/csrc`")
    return got


def ptr(a):
    """float64 pointer of a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(_P)


def f64(a, ndim=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if ndim == 2 and a.ndim == 1:
        a = a.reshape(-1, 1)
    return a


class Context:
    """One device + one HIP stream + the device-resident buffers of the hot path."""

    def __init__(self, device=0):
        self.lib = load()
        h = _c_vp()
        rc = self.lib.gps_ctx_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise GpsError(f"gps_ctx_create(device={device}) failed: "
                           f"{self.lib.gps_last_error(None).decode()}")
        self.h = h
        self.device = device
        # which GP object's data the device currently holds, per kind ("full" / "fitc")
        self.resident = {}

    def check(self, rc, what):
        if rc == 0:
            return
        msg = self.lib.gps_last_error(self.h).decode()
        if rc > 0:
            raise NotPositiveDefinite(rc, f"{what}: {msg}")
        raise GpsError(f"{what} failed ({rc}): {msg}")

    def call(self, name, *args):
        self.check(getattr(self.lib, name)(self.h, *args), name)

    def close(self):
        if getattr(self, "h", None):
            self.lib.gps_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- profiling
    def prof(self, on=True):
        self.call("gps_prof_enable", 1 if on else 0)

    def prof_collect(self):
        import json
        buf = ctypes.create_string_buffer(1 << 16)
        self.call("gps_prof_collect", buf, len(buf))
        return json.loads(buf.value.decode())

    def phases(self, on=True):
        """Phase timing of the FITC forward on its production schedule (gps_phase_enable)."""
        self.call("gps_phase_enable", 1 if on else 0)

    def phase_collect(self):
        """{"phases": {name: {count, ms}}, "allreduce": [[bytes, ms], ...]} since the last
        collect (gps_phase_collect)."""
        import json
        buf = ctypes.create_string_buffer(1 << 20)
        self.call("gps_phase_collect", buf, len(buf))
        return json.loads(buf.value.decode())

    def set_overlap(self, on=True):
        """Run the factorisation's off-critical-path GEMMs on a second stream."""
        self.call("gps_ctx_set_option", GPS_OPT_OVERLAP, 1 if on else 0)

    def set_tiny_gemm(self, on=True):
        """The small kernel (16/32-blocks per wave, K split across a workgroup's waves) for
        the GEMMs at the bottom of the recursion (default) or the 64-tile split-K path
        (process-wide)."""
        self.call("gps_ctx_set_option", GPS_OPT_TINY_GEMM, 1 if on else 0)

    def set_gram_reg(self, on=True):
        """Gram kernels (process-wide): True / 2 (default) the d = 8, 16 builds on the matrix
        cores (the reference's expansion, centred), d = 1 on the register-resident kernel; 1 the
        register-resident direct-difference kernels (bitwise equal to 0); False / 0 the
        LDS-column kernel."""
        v = on if isinstance(on, int) and not isinstance(on, bool) else (2 if on else 0)
        self.call("gps_ctx_set_option", GPS_OPT_GRAM_REG, v)

    def set_graphs(self, on=True):
        """Replay the recursive factorisation from a captured hipGraph (default) or launch
        it eagerly."""
        self.call("gps_ctx_set_option", GPS_OPT_GRAPH, 1 if on else 0)

    def set_ar_chunks(self, chunks):
        """Sharded FITC: B's all-reduce in this many row blocks overlapped with the SYRK
        (GPS_OPT_AR_CHUNKS, default 4; 1 = one all-reduce after the SYRK)."""
        self.call("gps_ctx_set_option", GPS_OPT_AR_CHUNKS, int(chunks))

    def set_dag(self, on=True, tiles=None):
        """The persistent factorisation of the bottom diagonal blocks (GPS_OPT_DAG, default on)
        and its largest block in 128-tiles (GPS_OPT_DAG_TILES)."""
        self.call("gps_ctx_set_option", GPS_OPT_DAG, 1 if on else 0)
        if tiles is not None:
            self.call("gps_ctx_set_option", GPS_OPT_DAG_TILES, int(tiles))

    def set_pred_pre(self, on=True):
        """FITC: form the q_i = ||Lm^-1 k_i||^2 columns that need only the top-level Lm11^-1
        during Lm's factorisation (default), or the whole pass after it."""
        self.call("gps_ctx_set_option", GPS_OPT_PRED_PRE, 1 if on else 0)

    def synchronize(self):
        self.call("gps_ctx_synchronize")

    def stats(self):
        """{graphs, graph_cap, graph_overflow, device_bytes, graph_dropped, graph_evicted}
        (gps_ctx_stats)."""
        out = np.zeros(GPS_N_STATS, np.int64)
        rc = self.lib.gps_ctx_stats(self.h, out.ctypes.data_as(ctypes.c_void_p), GPS_N_STATS)
        self.check(0 if rc >= 0 else rc, "gps_ctx_stats")
        return dict(zip(("graphs", "graph_cap", "graph_overflow", "device_bytes", "graph_dropped",
                         "graph_evicted"), (int(v) for v in out)))

    def comm_info(self):
        """(nranks, rank, kind) of the context's communicator as the library sees it: RCCL's own
        ncclCommCount / ncclCommUserRank, the in-process group's, or (1, 0, "none")."""
        n, r, k = _c_int(), _c_int(), _c_int()
        self.call("gps_comm_info", ctypes.byref(n), ctypes.byref(r), ctypes.byref(k))
        return n.value, r.value, COMM_KINDS.get(k.value, str(k.value))

    def set_stream(self, stream_handle):
        self.call("gps_ctx_set_stream", _c_vp(stream_handle))


_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        dev = int(os.environ.get("GPSCORE_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        _default_ctx = Context(dev)
    return _default_ctx
