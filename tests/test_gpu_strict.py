"""The strict-radiance build (_build/librtw_strict.so, RTW_STRICT_RADIANCE)
against the oracle to the LAST BIT.

The product build reaches the reference's radiance within a few ulps: every
path decision is the reference's, but the recursion of color()
(RayTracingWeekend.cpp:45-160) is folded forward and the radiance-only
quotients are reordered (RTW_RADIANCE_FAST / RTW_RADIANCE_RCP, rtw_device.h).
The strict build keeps the reference's expressions and folds each path's
factors inside-out at its end, ((attenuation * scattering_pdf) * color) /
pdf_val (:129-132) and attenuation * color (:107), as the recursion returns
them.  What is left between the device and glibc is the libm: the device's
azimuth sincos, texture sine, media log and schlick pow5 (rtw_math.h; within
an ulp of glibc's, tests/test_sincos.py).  So the checker here is the oracle
built with those same functions (oracle/_ref/librtw_oracle_devlibm.so,
oracle/devlibm.cpp) -- the plain-C restatement pinned bit for bit to the
reference's renders (tests/test_oracle.py) with only its libm calls swapped
-- and the per-pixel sums must be EQUAL (np.array_equal), with equal
device-counted traversals, on every scene family, flat and BVH.
"""
import ctypes as C

import numpy as np
import pytest

from oracle_lib import ROOT

pytestmark = pytest.mark.gpu

DEVLIBM_SO = ROOT / "oracle" / "_ref" / "librtw_oracle_devlibm.so"

# scene, nx, ny, spp, depth, bvh
CASES = [
    ("cornell_box", 32, 32, 4, 50, False),
    ("cornell_box", 24, 24, 3, 100, False),
    ("random_balls", 48, 32, 4, 50, False),
    ("random_balls", 48, 32, 4, 50, True),
    ("dielectric", 32, 16, 4, 50, False),
    ("light_sample", 32, 16, 4, 50, False),
    ("book2_final", 24, 24, 2, 50, True),
    ("nested", 24, 24, 4, 50, False),
]


@pytest.fixture(scope="module")
def strict(built):
    from raytracingweekend_amd import _abi, build
    from conftest import stale
    L = _abi.load_library(build.STRICT_LIB)
    # the strict library's own build id against the sources' with its flags
    stale(build.STRICT_LIB.name, L.rtw_build_id().decode(), build.build_id(["-DRTW_STRICT_RADIANCE=1"]))
    if L.rtw_device_count() < 1:
        pytest.fail("no GPU visible to the HIP runtime")
    return L


@pytest.fixture(scope="module")
def devlibm_oracle(built):
    from raytracingweekend_amd import _abi
    assert DEVLIBM_SO.exists(), "oracle/_ref/librtw_oracle_devlibm.so is built by build_all (oracle/Makefile port)"
    L = C.CDLL(str(DEVLIBM_SO))
    L.rtw_oracle_render_strided.restype = C.c_int
    L.rtw_oracle_render_strided.argtypes = [C.POINTER(_abi.rtw_scene_desc), C.POINTER(_abi.rtw_camera_desc),
                                            C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.c_int, C.c_uint64, C.c_int, C.c_void_p, C.POINTER(C.c_uint64)]
    return L


def strict_render(L, scene, nx, ny, spp, depth, seed, bvh):
    """rtw_scene_builtin -> rtw_scene_upload -> rtw_render_accumulate through
    the strict library's own C ABI; returns (sums, traversals, kernel)."""
    from raytracingweekend_amd import _abi
    d = C.POINTER(_abi.rtw_scene_desc)()
    _abi.check(L.rtw_scene_builtin(scene.encode(), nx / ny, int(bvh), C.byref(d)), "strict builtin")
    h = C.c_void_p()
    try:
        assert L.rtw_scene_upload(0, d, C.byref(h)) == 0, L.rtw_last_error()
        info = _abi.rtw_scene_info()
        assert L.rtw_scene_query(h, C.byref(info)) == 0
        acc = np.zeros(nx * ny * 3)
        prm = _abi.rtw_render_params(nx=nx, ny=ny, spp=spp, max_depth=depth, seed=seed, row_step=1)
        st = _abi.rtw_stats()
        assert L.rtw_render_accumulate(h, C.byref(d.contents.camera), C.byref(prm), acc.ctypes.data_as(C.c_void_p),
                                       C.byref(st)) == 0, L.rtw_last_error()
        return acc, st.segments, info.as_dict()["kernel"]
    finally:
        if h:
            L.rtw_scene_free(h)
        L.rtw_scene_desc_free(d)


def oracle_render(O, scene, nx, ny, spp, depth, seed):
    from raytracingweekend_amd.render import SceneDesc
    sd = SceneDesc(scene, nx / ny)  # the oracle walks the flat list (BVH = flat list, bit for bit)
    out = np.zeros(nx * ny * 3)
    seg = C.c_uint64(0)
    assert O.rtw_oracle_render_strided(sd.ptr, C.byref(sd.camera), nx, ny, 0, 1, ny, 0, spp, depth, seed, 0,
                                       out.ctypes.data_as(C.c_void_p), C.byref(seg)) == 0
    return out, seg.value


@pytest.mark.parametrize("scene,nx,ny,spp,depth,bvh", CASES,
                         ids=[f"{c[0]}_{c[1]}x{c[2]}x{c[3]}_d{c[4]}" + ("_bvh" if c[5] else "") for c in CASES])
def test_strict_build_equals_devlibm_oracle_bit_for_bit(strict, devlibm_oracle, scene, nx, ny, spp, depth, bvh):
    seed = 7
    got, seg, kernel = strict_render(strict, scene, nx, ny, spp, depth, seed, bvh)
    want, oseg = oracle_render(devlibm_oracle, scene, nx, ny, spp, depth, seed)
    assert kernel.startswith("k_persist<"), kernel  # the strict build folds in k_persist
    assert seg == oseg, "device-counted traversals differ from the oracle's"
    diff = np.flatnonzero(got != want)
    assert diff.size == 0, (f"{diff.size} of {got.size} channel sums differ; first at {diff[:4]}: "
                            f"{got[diff[:4]]} vs {want[diff[:4]]}")


def test_product_build_is_within_ulps_of_strict(strict):
    """The product build (forward fold, fewer divisions) against the strict
    one on the same paths: equal traversals, sums within 1e-12 relative --
    the reorderings move radiance by ulps, never a path."""
    from raytracingweekend_amd.render import DeviceScene, SceneDesc
    nx, ny, spp, depth, seed = 32, 32, 4, 50, 7
    got, seg, _ = strict_render(strict, "cornell_box", nx, ny, spp, depth, seed, False)
    ds = DeviceScene(SceneDesc("cornell_box", nx / ny))
    try:
        fast, st = ds.render_accumulate(nx, ny, spp, depth, seed)
    finally:
        ds.close()
    assert st["segments"] == seg
    assert np.allclose(fast, got, rtol=1e-12, atol=1e-300)
