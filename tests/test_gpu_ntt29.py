"""GPU: the opt-in radix-2^29 NTT kernels (csrc/ntt29.hip, STARK_NTT29=1) against the oracle at every
pass plan 2^2..2^20 and through the LDE's sparse first pass.  The switch is read once per process, so
the check runs as one child process (tools/check_ntt29.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_ntt29_parity():
    env = dict(os.environ, STARK_NTT29="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_ntt29.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ntt29 parity: ok" in r.stdout, r.stdout + r.stderr
