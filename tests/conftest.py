import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")


def golden_names(prefix=""):
    return sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def theta_of(g):
    """(log_sf2, log_ell, log_sn2, kind) of a golden case."""
    if "theta" in g:
        t = g["theta"]
        return (float(t[0]), float(t[1]), float(t[2])), str(g.get("kern", "ARD"))
    return (float(g["log_sf2"]), g["log_ell"], float(g["log_sn2"])), "ARD"


def nrel(a, b):
    """normwise relative error max|a-b| / max|b|."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.fixture(scope="session")
def gpu_ctx():
    import gpscore
    return gpscore.Context(0)


@pytest.fixture(scope="session", autouse=True)
def library_is_head_build():
    """Every session (CPU or GPU) runs against the library built from the checked-out csrc/:
    gps_build_id must equal the hash of these sources (gpscore/buildid.py), so a passing record
    names HEAD's build and not a stale or foreign binary."""
    from gpscore import _lib
    if os.path.exists(_lib.LIB_PATH):
        _lib.check_build_id()


# ------------------------------------------------------------------ parity floors record
# Every measured-floor comparison (the BASELINE configs, the shard splits, the CP.R surfaces)
# records {test: {output: [gpu-vs-reference error, measured floor, absolute cap]}}; the session
# writes them to $GPS_PARITY_FLOORS (default gpurun_out/parity_floors.json) so the margins are
# visible outside pytest's captured output (committed as profiles/r3_parity_floors.json).
PARITY_FLOORS = {}


def record_floors(test, errs, floors, caps):
    rec = PARITY_FLOORS.setdefault(test, {})
    for k, e in errs.items():
        rec[k] = [float(e), float(floors.get(k, float("nan"))), float(caps.get(k, float("nan")))]


def pytest_sessionfinish(session, exitstatus):
    if not PARITY_FLOORS:
        return
    import json
    path = os.environ.get("GPS_PARITY_FLOORS", os.path.join(ROOT, "gpurun_out", "parity_floors.json"))
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        old = {}
        if os.path.exists(path):
            with open(path) as f:
                old = json.load(f)
        old.update(PARITY_FLOORS)
        with open(path, "w") as f:
            json.dump(old, f, indent=1, sort_keys=True)
    except OSError:
        pass
