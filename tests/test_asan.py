"""Host-side AddressSanitizer pass over the C-ABI (SURVEY.md §5 "race detection / sanitizers"):
libgpscore_asan.so (`make -C <pkg>/csrc asan`: host code under -fsanitize=address, device code
unchanged) driven by tools/asan_check.py in a subprocess with the ASan runtime preloaded."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd")
ASAN_LIB = os.path.join(PKG, "gpscore", "libgpscore_asan.so")
ASAN_RT = "/opt/rocm/lib/llvm/lib/clang/22/lib/linux/libclang_rt.asan-x86_64.so"
HSA_RT = "/opt/rocm/lib/libhsa-runtime64.so.1"


def _run(mode):
    if not os.path.exists(ASAN_LIB):
        pytest.skip("libgpscore_asan.so not built (make -C <pkg>/csrc asan; __graft_entry__.build does)")
    rt = ASAN_RT
    if not os.path.exists(rt):
        rt = subprocess.run(["/opt/rocm/bin/hipcc", "-print-file-name=libclang_rt.asan-x86_64.so"],
                            capture_output=True, text=True).stdout.strip()
    env = dict(os.environ)
    # The HSA runtime goes ahead of the ASan runtime: the ASan runtime's own interceptor of
    # hsa_amd_memory_pool_allocate (its GPU-ASan support, which needs XNACK-enabled device code)
    # ran out of memory at HIP's first device allocation on every pool box (r4:
    # gpurun_out/asan_dev_a1.err); preloaded first, libhsa-runtime64 keeps its own definition of the
    # hsa_* symbols for HIP, while malloc / free and the other host interceptors stay ASan's (the
    # first preloaded library that defines them).  That order needs verify_asan_link_order=0.
    pre = [HSA_RT] if os.path.exists(HSA_RT) else []
    env["LD_PRELOAD"] = " ".join(pre + [rt] + ([env["LD_PRELOAD"]] if env.get("LD_PRELOAD") else []))
    env["ASAN_OPTIONS"] = ("detect_leaks=0:abort_on_error=1:halt_on_error=1"
                           + (":verify_asan_link_order=0" if pre else ""))
    env["GPSCORE_LIB"] = ASAN_LIB
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asan_check.py"), mode],
                       env=env, capture_output=True, text=True, timeout=240)
    if (p.returncode != 0 and "out of memory" in p.stderr
            and "hsa_amd_memory_pool_allocate" in p.stderr):
        # the ASan runtime's own interceptor of HSA device allocations (its GPU-ASan support)
        # failed before our code ran: an environment limit of the box (seen on some pool
        # boxes, not others), not a finding in the host code under test
        pytest.skip("ASan runtime's HSA device-allocation interceptor ran out of memory on this box")
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "AddressSanitizer" not in p.stderr, p.stderr[-3000:]
    return p.stdout


def test_asan_null_context_paths():
    """Every entry point with a NULL context, and context creation without a device."""
    assert "entry points rejected" in _run("null")


@pytest.mark.gpu
def test_asan_device_argument_validation():
    """A real context: invalid arguments to every entry point, then small valid fits, predicts,
    gradients, block-LOO, FITC, compat and surface calls — all under host ASan."""
    assert "valid paths clean" in _run("device")
