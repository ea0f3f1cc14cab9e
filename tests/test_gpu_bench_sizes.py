"""GPU parity at the benchmarked sizes (BASELINE.json configs).

The bench renders 800x800 (T, C4), 1200x800 (C2, C3) and 1600x1600 (C5)
images with up to 4096 samples per pixel; the RNG key of a sample is (seed,
pixel id up to nx*ny-1, sample id up to spp-1) (rtw_path_seed).  The oracle is
far too slow for whole images at those sizes, but every pixel is independent,
so the kernels are checked on BANDS of the full-size images: a few rows spread
over the image (row_begin / row_step of rtw_render_params) and the LAST samples
of the pixel's range (the top of the key space), against the oracle on the
same rows and samples -- and, for T, C2, C3 and C5, on the WHOLE full-size
image at the last sample of every pixel.  Tolerance as tests/test_gpu_parity.py: 1e-4 per
canvas channel (north star), equal device-counted traversals.
"""
import numpy as np
import pytest

from oracle_lib import finalize_np, oracle_sums

pytestmark = pytest.mark.gpu

TOL = 1e-4

# name, scene, nx, ny, spp (total), samples at the top of the range, bvh, rows (begin, step)
BANDS = [
    ("T", "cornell_box", 800, 800, 1024, 8, False, (3, 97)),
    ("C4", "cornell_box", 800, 800, 4096, 4, False, (41, 181)),
    ("C2", "random_balls", 1200, 800, 256, 4, False, (5, 131)),
    ("C3", "random_balls", 1200, 800, 1024, 4, True, (7, 149)),
    ("C5", "book2_final", 1600, 1600, 4096, 2, True, (401, 400)),
]


@pytest.fixture(scope="module")
def gpu(built):
    from raytracingweekend_amd import render
    if render.device_count() < 1:
        pytest.fail("no GPU visible to the HIP runtime")
    return render


def band_rows(ny, begin, step):
    return list(range(begin, ny, step))


def oracle_band(sd, nx, ny, spp, depth, seed, rows, s_begin, s_count):
    acc = np.zeros(nx * ny * 3)
    seg = 0
    for r in rows:
        a, s = oracle_sums(sd, nx, ny, spp, depth, seed, rows=(r, 1), spp_begin=s_begin, spp_count=s_count)
        acc += a  # rows are disjoint; other rows stay 0
        seg += s
    return acc, seg


@pytest.mark.parametrize("name,scene,nx,ny,spp,cnt,bvh,rows", BANDS, ids=[b[0] for b in BANDS])
def test_band_matches_oracle(gpu, name, scene, nx, ny, spp, cnt, bvh, rows):
    depth, seed = 50, 0
    sd = gpu.SceneDesc(scene, nx / ny, use_bvh=bvh)
    ds = gpu.DeviceScene(sd)
    try:
        acc, st = ds.render_accumulate(nx, ny, spp, depth, seed, spp_begin=spp - cnt, spp_count=cnt,
                                       row_begin=rows[0], row_step=rows[1])
    finally:
        ds.close()
    rlist = band_rows(ny, *rows)
    ref, seg = oracle_band(gpu.SceneDesc(scene, nx / ny), nx, ny, spp, depth, seed, rlist, spp - cnt, cnt)
    assert st["samples"] == len(rlist) * nx * cnt
    assert st["segments"] == seg, "device-counted traversals differ from the oracle's"
    sel = np.zeros((ny, nx * 3), dtype=bool)
    sel[rlist] = True
    sel = sel.reshape(-1)
    assert not acc[~sel].any(), "rows outside the band were written"
    d = np.abs(finalize_np(acc[sel], cnt) - finalize_np(ref[sel], cnt))
    assert np.all(np.isfinite(acc[sel]))
    assert d.max() <= TOL, f"{name}: max per-channel diff {d.max()}"


# whole images at the bench resolution, the LAST sample of each pixel (the
# oracle renders them in seconds; Book 2's 2.56 M paths would take minutes)
WHOLE = [
    ("T", "cornell_box", 800, 800, 1024, False),
    ("C2", "random_balls", 1200, 800, 256, False),
    ("C3", "random_balls", 1200, 800, 1024, True),
]


@pytest.mark.parametrize("name,scene,nx,ny,spp,bvh", WHOLE, ids=[w[0] for w in WHOLE])
def test_whole_image_last_sample_matches_oracle(gpu, name, scene, nx, ny, spp, bvh):
    """Every pixel of the full-size image (not a band), at the top of the
    sample range: equal device-counted traversals, canvas within 1e-4, and
    the quantised (PPM) channels equal except at rounding boundaries."""
    depth, seed = 50, 0
    sd = gpu.SceneDesc(scene, nx / ny, use_bvh=bvh)
    ds = gpu.DeviceScene(sd)
    try:
        acc, st = ds.render_accumulate(nx, ny, spp, depth, seed, spp_begin=spp - 1, spp_count=1)
    finally:
        ds.close()
    ref, seg = oracle_sums(gpu.SceneDesc(scene, nx / ny), nx, ny, spp, depth, seed, spp_begin=spp - 1, spp_count=1)
    assert st["samples"] == nx * ny
    assert st["segments"] == seg, "device-counted traversals differ from the oracle's"
    c_gpu, c_ref = finalize_np(acc, 1), finalize_np(ref, 1)
    assert np.all(np.isfinite(c_gpu))
    d = np.abs(c_gpu - c_ref)
    assert d.max() <= TOL, f"{name}: max per-channel diff {d.max()}"
    q_gpu = (np.float64(np.float32(255.99)) * c_gpu).astype(np.int64)
    q_ref = (np.float64(np.float32(255.99)) * c_ref).astype(np.int64)
    assert (q_gpu != q_ref).sum() <= max(1, d.size // 10000)


@pytest.mark.parametrize("phase", range(4), ids=[f"rows{k}mod4" for k in range(4)])
def test_whole_C5_image_last_sample_matches_oracle(gpu, phase):
    """The whole C5 image (Book-2 final 1600x1600, BVH on the GPU, the flat
    list in the oracle) at the last of its 4096 samples, every pixel compared:
    four interleaved row sets (rows j = phase mod 4) so each part is ~15 s of
    the oracle over the box's host threads.  Media (hittable.h:420-489),
    Perlin marble (noise.h:74-151), moving spheres and the box ground: equal
    device-counted traversals, canvas within 1e-4, PPM channels equal but for
    rounding boundaries."""
    nx, ny, spp, depth, seed = 1600, 1600, 4096, 50, 0
    sd = gpu.SceneDesc("book2_final", 1.0, use_bvh=True)
    ds = gpu.DeviceScene(sd)
    try:
        acc, st = ds.render_accumulate(nx, ny, spp, depth, seed, spp_begin=spp - 1, spp_count=1, row_begin=phase,
                                       row_step=4)
    finally:
        ds.close()
    rows = list(range(phase, ny, 4))
    ref, seg = oracle_sums(gpu.SceneDesc("book2_final", 1.0), nx, ny, spp, depth, seed, rows=(phase, len(rows), 4),
                           spp_begin=spp - 1, spp_count=1)
    assert st["samples"] == nx * len(rows)
    assert st["segments"] == seg, "device-counted traversals differ from the oracle's"
    sel = np.zeros((ny, nx * 3), dtype=bool)
    sel[rows] = True
    sel = sel.reshape(-1)
    assert not acc[~sel].any(), "rows outside the set were written"
    c_gpu, c_ref = finalize_np(acc[sel], 1), finalize_np(ref[sel], 1)
    assert np.all(np.isfinite(c_gpu))
    d = np.abs(c_gpu - c_ref)
    assert d.max() <= TOL, f"C5 rows {phase} mod 4: max per-channel diff {d.max()}"
    q_gpu = (np.float64(np.float32(255.99)) * c_gpu).astype(np.int64)
    q_ref = (np.float64(np.float32(255.99)) * c_ref).astype(np.int64)
    assert (q_gpu != q_ref).sum() <= max(1, d.size // 10000)


def test_multi_pass_at_T_resolution(gpu, monkeypatch):
    """A band of the T image forced through several passes (pass budget of 3
    samples per pixel: radiance buffer reused, per-pixel running sums carried
    across passes) equals the one-pass render bit for bit."""
    nx, ny, spp, depth, cnt = 800, 800, 1024, 50, 8
    rows = (3, 97)
    npix = len(band_rows(ny, *rows)) * nx
    sd = gpu.SceneDesc("cornell_box", 1.0)
    ds = gpu.DeviceScene(sd)
    try:
        one, st1 = ds.render_accumulate(nx, ny, spp, depth, 0, spp_begin=spp - cnt, spp_count=cnt,
                                        row_begin=rows[0], row_step=rows[1])
        monkeypatch.setenv("RTW_PASS_SAMPLES", str(npix * 3))
        many, st3 = ds.render_accumulate(nx, ny, spp, depth, 0, spp_begin=spp - cnt, spp_count=cnt,
                                         row_begin=rows[0], row_step=rows[1])
    finally:
        ds.close()
    assert st1["launches_intersect"] == 1 and st3["launches_intersect"] == 3
    assert st1["segments"] == st3["segments"]
    assert np.array_equal(one, many)


def test_full_T_image_statistics(gpu):
    """The whole T image at 64 of its 1024 samples: every pixel rendered
    (sample counts, finite radiance), sample shards [0, 32) + [32, 64) equal to
    [0, 64) within fp64 reassociation, and segments per sample where the
    survey measured the reference (5.227)."""
    nx, ny, spp, depth = 800, 800, 1024, 50
    sd = gpu.SceneDesc("cornell_box", 1.0)
    ds = gpu.DeviceScene(sd)
    try:
        full, st = ds.render_accumulate(nx, ny, spp, depth, 0, spp_begin=0, spp_count=64)
        a = np.zeros_like(full)
        ds.render_accumulate(nx, ny, spp, depth, 0, spp_begin=0, spp_count=32, accum=a)
        ds.render_accumulate(nx, ny, spp, depth, 0, spp_begin=32, spp_count=32, accum=a)
    finally:
        ds.close()
    assert st["samples"] == nx * ny * 64
    assert np.all(np.isfinite(full))
    assert np.allclose(a, full, rtol=1e-12, atol=1e-12)
    assert 5.0 < st["segments"] / st["samples"] < 5.5


def test_render_multi_one_gpu_is_bit_exact(gpu):
    """rtw_render_multi with one device (RCCL communicator of one rank) gives
    exactly rtw_render_accumulate's accumulator, host and device pointers."""
    import torch
    nx, ny, spp, depth = 64, 48, 6, 50
    sd = gpu.SceneDesc("cornell_box", nx / ny)
    ds = gpu.DeviceScene(sd)
    try:
        ref, st_ref = ds.render_accumulate(nx, ny, spp, depth, 4)
        got, st = gpu.render_multi([ds], nx, ny, spp, depth, 4)
        assert np.array_equal(got, ref)
        assert st["segments"] == st_ref["segments"] and st["samples"] == st_ref["samples"]
        dev = torch.full((nx * ny * 3,), 0.5, dtype=torch.float64, device="cuda:0")
        gpu.render_multi([ds], nx, ny, spp, depth, 4, accum=dev)
        assert np.array_equal(dev.cpu().numpy(), ref + 0.5)
        # a sample sub-range and a row subset, as rtw_render_accumulate takes them
        part, _ = ds.render_accumulate(nx, ny, spp, depth, 4, spp_begin=2, spp_count=3, row_begin=1, row_step=2)
        got2, _ = gpu.render_multi([ds], nx, ny, spp, depth, 4, spp_begin=2, spp_count=3, row_begin=1, row_step=2)
        assert np.array_equal(got2, part)
    finally:
        gpu.lib().rtw_release_communicators()
        ds.close()


def test_device_quantize_and_ppm_bytes(gpu, tmp_path):
    """rtw_quantize_canvas_device (int(255.99f * c) on the GPU) equals the host
    writer's quantisation, and the quantized writer emits the same bytes as
    rtw_write_ppm (RayTracingWeekend.cpp:257-276)."""
    import torch
    nx, ny, spp = 40, 30, 4
    sd = gpu.SceneDesc("cornell_box", nx / ny)
    ds = gpu.DeviceScene(sd)
    try:
        acc = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda:0")
        ds.render_accumulate(nx, ny, spp, 50, seed=2, accum=acc)
        canvas = ds.finalize_device(acc, nx, ny, spp)
        canvas[:4] = torch.tensor([float("nan"), -0.5, 1.0, 0.999], dtype=torch.float64)
        q = ds.quantize_device(canvas, nx, ny).cpu().numpy()
    finally:
        ds.close()
    c = canvas.cpu().numpy()
    gpu.write_ppm(tmp_path / "a.ppm", c, nx, ny)
    gpu.write_ppm_quantized(tmp_path / "b.ppm", q, nx, ny)
    assert (tmp_path / "a.ppm").read_bytes() == (tmp_path / "b.ppm").read_bytes()
    assert q[0] == -2147483648 and q[1] == -127 and q[2] == 255 and q[3] == 255  # int() truncates toward 0


def test_scene_query_names_the_launched_kernel(gpu):
    sd = gpu.SceneDesc("cornell_box", 1.0)
    ds = gpu.DeviceScene(sd)
    try:
        info = ds.query()
    finally:
        ds.close()
    assert info["kernel"].startswith("k_persist_sort<")
    assert info["build_id"] == gpu.build_id() and info["build_id"] != "unknown"
    assert info["n_world_runs"] >= 1 and info["shade_lds_bytes"] > 0


def test_multi_pass_at_C5_resolution(gpu, monkeypatch):
    """The whole C5 image (Book-2 final, 1600x1600, BVH) at 16 of its 4096
    samples, forced through 4 passes of 4 samples per pixel (the full config
    runs 10 passes of 2^30 samples): every pixel rendered (sample counts,
    finite radiance), traversals per sample where the one-pass render and the
    bench put them (~5.62), and the multi-pass accumulator bit-identical to the
    one-pass one (per-pixel running sums carried across passes in sample
    order, RayTracingWeekend.cpp:235-239)."""
    nx, ny, spp, depth, cnt = 1600, 1600, 4096, 50, 16
    sd = gpu.SceneDesc("book2_final", 1.0, use_bvh=True)
    ds = gpu.DeviceScene(sd)
    try:
        one, st1 = ds.render_accumulate(nx, ny, spp, depth, 0, spp_begin=spp - cnt, spp_count=cnt)
        monkeypatch.setenv("RTW_PASS_SAMPLES", str(nx * ny * 4))
        many, st4 = ds.render_accumulate(nx, ny, spp, depth, 0, spp_begin=spp - cnt, spp_count=cnt)
    finally:
        ds.close()
    assert st1["launches_intersect"] == 1 and st4["launches_intersect"] == 4
    assert st1["samples"] == st4["samples"] == nx * ny * cnt
    assert st1["segments"] == st4["segments"]
    assert 5.4 < st4["segments"] / st4["samples"] < 5.85
    assert np.all(np.isfinite(many))
    assert np.array_equal(one, many)
    lum = many.reshape(-1, 3).sum(axis=1)
    assert (lum > 0).mean() > 0.5  # a lit image, not a zeroed buffer


def test_render_multi_rejects_bad_handles_and_accumulators(gpu):
    """rtw_render_multi: two handles on one device are refused, and so is a
    device accumulator that is not device memory of handles[0]'s GPU
    (rtw_render_accumulate likewise)."""
    import ctypes as C
    import torch
    from raytracingweekend_amd import _abi
    nx, ny, spp = 16, 16, 2
    sd = gpu.SceneDesc("cornell_box", 1.0)
    a, b = gpu.DeviceScene(sd), gpu.DeviceScene(sd)
    L = gpu.lib()
    try:
        with pytest.raises(_abi.RtwError, match="two handles on one device"):
            gpu.render_multi([a, b], nx, ny, spp, 10)
        hs = (C.c_void_p * 1)(a.handle.value)
        prm = _abi.rtw_render_params(nx=nx, ny=ny, spp=spp, max_depth=10, row_step=1, accum_on_device=1)
        host = np.zeros(nx * ny * 3)
        assert L.rtw_render_multi(1, hs, C.byref(sd.camera), C.byref(prm), host.ctypes.data_as(C.c_void_p),
                                  None) == -1
        assert b"not device or managed memory" in L.rtw_last_error()
        assert L.rtw_render_accumulate(a.handle, C.byref(sd.camera), C.byref(prm), host.ctypes.data_as(C.c_void_p),
                                       None) == -1
        assert b"not device or managed memory" in L.rtw_last_error()
        prm.accum_on_device, prm.precision = 0, 7
        assert L.rtw_render_accumulate(a.handle, C.byref(sd.camera), C.byref(prm), host.ctypes.data_as(C.c_void_p),
                                       None) == -1
        assert b"precision" in L.rtw_last_error()
        with pytest.raises(ValueError):
            a.render_accumulate(nx, ny, spp, 10, accum=torch.zeros(nx * ny * 3, dtype=torch.float64))
    finally:
        L.rtw_release_communicators()
        a.close()
        b.close()


def _loaded_hip_runtime():
    """The HIP runtime this process already runs (torch's, which librtw.so
    shares): the libamdhip64 mapped into the process, else the one the
    linker finds; skip when neither exists (no hard-coded soname)."""
    import ctypes as C
    import ctypes.util
    with open("/proc/self/maps") as f:
        for line in f:
            path = line.split()[-1] if line.strip() else ""
            if "libamdhip64.so" in path:
                return C.CDLL(path)
    name = ctypes.util.find_library("amdhip64")
    if not name:
        pytest.skip("the HIP runtime library cannot be located")
    return C.CDLL(name)


def test_managed_memory_accumulator(gpu):
    """A device accumulator in managed memory (hipMallocManaged) is accepted
    by rtw_render_accumulate and rtw_render_multi, and gives the same sums as
    a host accumulator."""
    import ctypes as C
    from raytracingweekend_amd import _abi
    hip = _loaded_hip_runtime()
    nx, ny, spp = 16, 12, 2
    n = nx * ny * 3
    sd = gpu.SceneDesc("cornell_box", nx / ny)
    a = gpu.DeviceScene(sd)
    L = gpu.lib()
    ptr = C.c_void_p()
    assert hip.hipMallocManaged(C.byref(ptr), C.c_size_t(n * 8), C.c_uint(1)) == 0  # hipMemAttachGlobal
    try:
        ref, _ = a.render_accumulate(nx, ny, spp, 10, seed=4)
        C.memset(ptr, 0, n * 8)
        prm = _abi.rtw_render_params(nx=nx, ny=ny, spp=spp, max_depth=10, seed=4, row_step=1, accum_on_device=1)
        _abi.check(L.rtw_render_accumulate(a.handle, C.byref(sd.camera), C.byref(prm), ptr, None), "managed")
        assert hip.hipDeviceSynchronize() == 0
        got = np.ctypeslib.as_array((C.c_double * n).from_address(ptr.value)).copy()
        assert np.array_equal(got, ref)
        C.memset(ptr, 0, n * 8)
        hs = (C.c_void_p * 1)(a.handle.value)
        _abi.check(L.rtw_render_multi(1, hs, C.byref(sd.camera), C.byref(prm), ptr, None), "managed multi")
        assert hip.hipDeviceSynchronize() == 0
        got = np.ctypeslib.as_array((C.c_double * n).from_address(ptr.value)).copy()
        assert np.array_equal(got, ref)
    finally:
        hip.hipFree(ptr)
        L.rtw_release_communicators()
        a.close()


@pytest.mark.skipif("not __import__('torch').cuda.is_available() or __import__('torch').cuda.device_count() < 2",
                    reason="needs two or more GPUs")
def test_render_multi_across_gpus_matches_one_gpu(gpu):
    """rtw_render_multi over every visible GPU (one host thread per device,
    ncclCommInitAll, grouped ncclReduce): equal to rtw_render_accumulate of the
    whole sample range within fp64 reassociation of the shard sums, host and
    device accumulators, with the same sample and traversal counts."""
    import torch
    n = min(torch.cuda.device_count(), 8)
    nx, ny, spp, depth = 96, 64, 2 * n + 1, 50
    sd = gpu.SceneDesc("cornell_box", nx / ny)
    scenes = [gpu.DeviceScene(sd, g) for g in range(n)]
    try:
        ref, st_ref = scenes[0].render_accumulate(nx, ny, spp, depth, 3)
        got, st = gpu.render_multi(scenes, nx, ny, spp, depth, 3)
        assert st["samples"] == st_ref["samples"] and st["segments"] == st_ref["segments"]
        assert np.allclose(got, ref, rtol=1e-13, atol=1e-13)
        dev = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda:0")
        gpu.render_multi(scenes, nx, ny, spp, depth, 3, accum=dev)
        assert np.allclose(dev.cpu().numpy(), ref, rtol=1e-13, atol=1e-13)
        with pytest.raises(ValueError):
            gpu.render_multi(scenes, nx, ny, spp, depth, 3,
                             accum=torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda:1"))
    finally:
        gpu.lib().rtw_release_communicators()
        for s in scenes:
            s.close()
