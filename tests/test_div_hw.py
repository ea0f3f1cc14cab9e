"""rtw_div.h's shared-divisor quotient (rcp_hw / div_hw), which the kernels
use for several quotients by one divisor, is bit-identical ON THE CARD to the
compiler's a / b inside its guarded operand range, and keeps quotients of
smaller numerators below 2^-599 (tests/cpp/div_hw_check.hip, 2^28 operand
pairs per class)."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "raytracingweekend_amd" / "_build" / "div_hw_check"


@pytest.mark.gpu
def test_shared_divisor_quotient_is_the_compilers_division():
    assert EXE.exists(), "build first: python -m raytracingweekend_amd.build"
    r = subprocess.run([str(EXE), "28"], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("mismatches 0 of") == 4


SQRT_EXE = ROOT / "raytracingweekend_amd" / "_build" / "sqrt_check"


@pytest.mark.gpu
def test_sqrt_core_is_the_compilers_sqrt():
    """rtw_div.h's sqrt_core (the compiler's sqrt sequence without its range
    scaling and class fixup) equals sqrt(x) bit for bit on the card for
    positive finite x >= 2^-766, and sqrt_w (core when the whole wave is in
    range) equals it for every bit pattern (tests/cpp/sqrt_check.hip)."""
    assert SQRT_EXE.exists(), "build first: python -m raytracingweekend_amd.build"
    r = subprocess.run([str(SQRT_EXE), "28"], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("mismatches 0 of") == 4
