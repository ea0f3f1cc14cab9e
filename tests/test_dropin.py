"""The reference's own scene code as a drop-in (tests/cpp/ref_dropin.cpp).

oracle/Makefile compiles the reference's UNCHANGED Scene/scene.h (where
/root/reference exists) against this repository's host headers and links it
with librtw.so; rtw_flatten (rtw/flatten.h) reads the reference scene through
its own accessors GetWorld / GetLights / GetCamera / GetRenderType /
GetBackgroundType (Scene/scene.h:24-31).

* CPU: every reference scene, flat and with BVHs, flattens to exactly the
  desc of rtw_scene_builtin (byte-equal arrays).
* GPU: the binary renders a reference scene through the C ABI, with the
  reference's main structure (RayTracingWeekend.cpp:195-289), and its PPM
  matches the oracle's for the same seed.  The binary was built here and
  travels with the tree like oracle/_ref/rtw_ref; the GPU box has no
  /root/reference and never reads it.
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "oracle" / "_ref" / "ref_dropin"
REF = Path("/root/reference/RayTracingWeekend/Scene/scene.h")


def _binary():
    if not BIN.exists():
        if REF.exists():
            pytest.fail("oracle/_ref/ref_dropin was not built although the reference is present")
        pytest.skip("ref_dropin is built only where /root/reference exists")
    return BIN


def test_reference_scene_h_flattens_like_the_builtins(built):
    r = subprocess.run([str(_binary()), "compare"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr
    assert r.stdout.count("identical") == 8


@pytest.mark.gpu
def test_reference_scene_renders_on_the_gpu(built, tmp_path):
    from oracle_lib import finalize_np, oracle_sums
    from raytracingweekend_amd.render import SceneDesc
    nx, ny, spp, depth, seed = 48, 48, 4, 50, 6
    out = tmp_path / "dropin.ppm"
    r = subprocess.run([str(_binary()), "render", "cornell_box", str(nx), str(ny), str(spp), str(depth), str(seed),
                        str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = np.array(out.read_text().split()[4:], dtype=np.int64)
    ref, _ = oracle_sums(SceneDesc("cornell_box", nx / ny), nx, ny, spp, depth, seed)
    c = finalize_np(ref, spp).reshape(ny, nx, 3)[::-1].reshape(-1)  # PPM rows top to bottom
    want = (np.float64(np.float32(255.99)) * c).astype(np.int64)
    assert (got != want).sum() <= 1, "PPM channels differ from the oracle's"
