"""Host-code sanitizer run: the kernels' host logic (tile cost models, grid sizing, shape
validation) built with ASan + UBSan on the host side and swept over every shape family -- on the CPU, no GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_kernel_host_code_under_asan_ubsan():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "host_asan", "build_and_run.sh")], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
