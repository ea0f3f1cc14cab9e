"""rtw_div.h's Markstein division (used for generate_canonical's divide in
every random draw on the device) is bit-identical to IEEE a / b: random,
rounding-midpoint and edge operands (tests/cpp/div_check.cpp)."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_markstein_division_is_ieee(tmp_path):
    exe = tmp_path / "div_check"
    # -mfma: hardware fma like the GPU's v_fma_f64 (glibc's fma is exact too)
    subprocess.run(["g++", "-std=c++17", "-O2", "-mfma", "-ffp-contract=off",
                    f"-I{ROOT / 'raytracingweekend_amd' / 'csrc'}", str(ROOT / "tests" / "cpp" / "div_check.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "canon cases" in r.stdout and "canon cases 0" not in r.stdout
    assert r.stdout.count("mismatches 0") == 2, r.stdout


def test_magic_number_division_is_exact(tmp_path):
    """rtw_div.h's udiv_fast (the sample id -> pixel / row decomposition of
    every camera sample) equals n / d on 32-bit operands: every divisor up to
    4 096, the image widths and pixel counts, powers of two and their
    neighbours, random divisors; n next to each multiple, at the range ends
    and random (tests/cpp/udiv_check.cpp); and mod_2p31m2 (the per-sample seed
    fold) equals x % (2^31 - 2) on 64-bit x."""
    exe = tmp_path / "udiv_check"
    subprocess.run(["g++", "-std=c++17", "-O2", f"-I{ROOT / 'raytracingweekend_amd' / 'csrc'}",
                    str(ROOT / "tests" / "cpp" / "udiv_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "2000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("mismatches 0") == 2 and "udiv cases 0 " not in r.stdout
