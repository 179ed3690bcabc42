"""CPU: div_const (csrc/cg_math.h) equals IEEE division for the constant divisors
the kernels use.  The exhaustive run (stride 1, all 2^32 floats, ~40 s per divisor)
is scripts/divchk.c; here a strided sample of ~1M inputs per divisor, which
includes zeros, denormals, infinities and NaNs."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def divchk(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    exe = tmp_path_factory.mktemp("divchk") / "divchk"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", "-o", str(exe),
                    os.path.join(ROOT, "scripts", "divchk.c"), "-lm"], check=True)
    return str(exe)


@pytest.mark.parametrize("b", ["3", "5", "9"])
def test_div_const_matches_ieee(divchk, b):
    r = subprocess.run([divchk, b, "4093"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert "mismatches=0" in r.stdout
