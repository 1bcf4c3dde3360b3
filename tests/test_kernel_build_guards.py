"""Build-level guards of the hand-written kernels (CPU only: hipcc cross-compiles for gfx950)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists(os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"))
                    and shutil.which("hipcc") is None, reason="hipcc not available")
def test_gemm4_accumulator_agprs_stay_asm_owned():
    """gemm4_k's accumulators live in AGPRs a[0:255] that only inline asm touches: no kernel
    variant may make the compiler write an AGPR (a spill into the accumulators) or spill to
    scratch (tools/check_agpr_ownership.py)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_agpr_ownership.py")],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
