"""an AddressSanitizer + UBSan build of the C++ host
code, exercised without a GPU (tools/asan): state-blob parsing on truncated,
bit-flipped and random blobs (gm_state_load must reject them before touching
any state), gm_gauss_from_cov on SPD / non-PD / NaN covariances, argument
validation of the create / run / diagnostics / BatchVector entry points, and
gm_init_positions into exactly sized buffers. Any out-of-bounds access or UB
aborts the driver."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "tools", "asan")


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="needs the ROCm toolchain")
def test_asan_host_checks():
    if not os.path.exists(os.path.join(ROOT, "general-mcmc_amd", "build", "gm_jit_headers.cpp.o")):
        pytest.skip("the main library build (make -C general-mcmc_amd) provides the kernel objects")
    r = subprocess.run(["make", "-s", "-C", ASAN, "-j8"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([os.path.join(ASAN, "build", "asan_host")], capture_output=True, text=True, timeout=600,
                       env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "asan host checks ok" in out, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
