"""The walks' e^{i t} (robustgrape_amd/csrc/grape_cis.hpp, round 6) on the host: built with hipcc as host
code (the same source the device code includes) and checked against x87 long double sinl / cosl --
at most 1 unit of 2^-52 absolute over |t| <= 1e5 (the library sincos's accuracy class), exact at 0."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and not shutil.which("hipcc"), reason="no hipcc")
def test_cis_fast_against_long_double(tmp_path):
    exe = str(tmp_path / "cis_check")
    subprocess.run([HIPCC, "-O2", "-ffp-contract=off", "-I" + os.path.join(ROOT, "robustgrape_amd", "csrc"),
                    os.path.join(ROOT, "tests", "c", "cis_check.cpp"), "-o", exe], check=True, capture_output=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    got = {k: float(v) for k, v in (line.split() for line in out.splitlines())}
    assert got["sin_err"] <= 1.0 and got["cos_err"] <= 1.0, got
    assert got["sin0"] == 0.0 and got["cos0"] == 1.0
