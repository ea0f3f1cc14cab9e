"""The BVH kernels' fp32 slab test (rtw_device.h make_slab_ray / slab32 /
t_lo32 / t_hi32) is conservative ON THE CARD: it never culls a box that the
real-arithmetic slab test keeps, over scene-sized rays, the whole magnitude
range the walks allow, exactly axis-parallel rays with origins on box planes,
and t ranges ending at the box's own entry / exit (tests/cpp/slab_check.hip,
2^26 rays per class, boxes placed on or within 2^-4 ... 2^-48 of the ray).
A culled real hit would change which primitives a BVH walk tests, so BVH
renders would stop equalling the flat list's."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "raytracingweekend_amd" / "_build" / "slab_check"


@pytest.mark.gpu
def test_fp32_slab_test_never_culls_a_real_hit():
    assert EXE.exists(), "build first: python -m raytracingweekend_amd.build"
    r = subprocess.run([str(EXE), "26"], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" misses 0 of ") == 4
