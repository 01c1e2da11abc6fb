"""Host-side checks of the engine's Go-math restatement (veneur_amd/csrc/gomath.h).

The kernels evaluate math.Asin (tdigest indexEstimate, merging_digest.go:240-243) in a
branch-free select form; it must equal the branchy restatement of Go 1.9's asin.go/atan.go
bit for bit.  Compiled for the host with hipcc (no GPU needed)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"), reason="hipcc absent")
def test_asin_select_form_bit_identical(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else "hipcc"
    exe = str(tmp_path / "asin_check")
    subprocess.check_call([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                           os.path.join(HERE, "native", "asin_check.cpp")])
    out = subprocess.run([exe, "1000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip().endswith("0 mismatches")
