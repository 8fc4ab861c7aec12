"""The C-ABI boundary on CPU: libgpscore.so loads and exports every symbol that
include/gpscore.h declares, and the ctypes binding covers all of them.
No compute calls (there is no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gpscore.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gps_\w+)\s*\(", txt)))


def test_header_declares_core_entry_points():
    syms = header_symbols()
    for s in ("gps_gram", "gps_potrf", "gps_potrs", "gps_diag_inv", "gps_full_fit",
              "gps_full_predict", "gps_scores", "gps_fitc_fit", "gps_fitc_grad", "gps_fitc_predict", "gps_full_blockloo", "gps_fitc_blockloo",
              "gps_comm_init", "gps_ctx_create", "gps_last_error"):
        assert s in syms


def test_library_exports_every_header_symbol():
    from gpscore import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} missing: run __graft_entry__.build()")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    from gpscore import _lib
    assert set(header_symbols()) == set(_lib.SIGNATURES), \
        set(header_symbols()) ^ set(_lib.SIGNATURES)
    lib = _lib.load()
    assert lib.gps_version() >= 100


def test_no_device_raises_loudly():
    """Without a GPU, creating a context must fail (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from gpscore import _lib
    with pytest.raises(_lib.GpsError):
        _lib.Context(0)


def test_rccl_info_names_the_loaded_rccl():
    """gps_rccl_info (no device needed): the RCCL version and the file that holds ncclAllReduce
    as the dynamic linker resolved it for this process — the bench's N > 1 line reports both
    (which RCCL actually ran).  The binding imports torch first in the test and
    bench processes, so the answer is either torch's bundled librccl or /opt/rocm's."""
    from gpscore import _lib
    v, path = _lib.rccl_info()
    assert v >= 20000, v  # NCCL_VERSION_CODE: major * 10000 + minor * 100 + patch
    assert "rccl" in os.path.basename(path), path
    assert os.path.exists(path), path
