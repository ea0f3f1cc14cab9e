"""Host-side Python API over the C ABI: the render loop of
RayTracingWeekend.cpp:195-289 (scene -> canvas -> PPM) with the per-pixel work
on the GPU.

    from raytracingweekend_amd import render
    canvas, stats = render.render("cornell_box", 400, 400, spp=64, max_depth=100)
    render.write_ppm("x64/1.ppm", canvas, 400, 400)

Multi-GPU (one process per GPU, torch.distributed over RCCL): see
raytracingweekend_amd.distributed.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import numpy as np

from . import _abi
from ._abi import check, lib


class SceneDesc:
    """A reference scene built with the host C++ scene API and flattened
    (rtw_scene_builtin).  Owns the library-allocated rtw_scene_desc."""

    def __init__(self, name: str, aspect: float, use_bvh: bool = False):
        self.name = name
        self.aspect = float(aspect)
        self.use_bvh = bool(use_bvh)
        p = C.POINTER(_abi.rtw_scene_desc)()
        check(lib().rtw_scene_builtin(name.encode(), self.aspect, int(use_bvh), C.byref(p)), "rtw_scene_builtin")
        self.ptr = p

    @property
    def desc(self) -> _abi.rtw_scene_desc:
        """A ctypes view of the library-owned descriptor.  The view keeps this
        SceneDesc (its owner) alive, so `SceneDesc(...).desc` of a temporary
        stays valid as long as the view does (the reference holds its scene
        graph by shared_ptr, Scene/scene.h:18-40)."""
        if not self.ptr:
            raise ValueError("SceneDesc is closed")
        view = self.ptr.contents
        view._rtw_owner = self
        return view

    @property
    def camera(self) -> _abi.rtw_camera_desc:
        """A view of the descriptor's camera; through its base view it keeps
        this SceneDesc alive (see `desc`)."""
        return self.desc.camera

    def close(self):
        if self.ptr:
            lib().rtw_scene_desc_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceScene:
    """A scene uploaded to one GPU (rtw_scene_upload)."""

    def __init__(self, scene: SceneDesc, device: int = 0):
        self.scene = scene
        self.device = device
        h = C.c_void_p()
        check(lib().rtw_scene_upload(device, scene.ptr, C.byref(h)), "rtw_scene_upload")
        self.handle = h

    def render_accumulate(self, nx: int, ny: int, spp: int, max_depth: int, seed: int = 0, *,
                          spp_begin: int = 0, spp_count: int = 0, row_begin: int = 0, row_step: int = 1,
                          accum=None, camera: Optional[_abi.rtw_camera_desc] = None,
                          collect_kernel_times: bool = False, wavefront_paths: int = 0, precision: str = "fp64"):
        """Add the per-pixel radiance sums of the selected samples into `accum`
        (a float64 numpy array of nx*ny*3, or a torch float64 CUDA tensor on
        this device).  precision "fp64" is the reference's arithmetic (parity
        mode); "fp32" the fast mode (statistical parity only).  Returns
        (accum, stats dict)."""
        if accum is None:
            accum = np.zeros(nx * ny * 3, dtype=np.float64)
        on_device = 0
        if isinstance(accum, np.ndarray):
            if accum.dtype != np.float64 or accum.size != nx * ny * 3 or not accum.flags["C_CONTIGUOUS"]:
                raise ValueError("accum must be a contiguous float64 array of nx*ny*3")
            ptr = accum.ctypes.data_as(C.c_void_p)
        else:  # torch tensor on the device
            import torch
            if accum.dtype != torch.float64 or accum.numel() != nx * ny * 3 or not accum.is_contiguous():
                raise ValueError("accum must be a contiguous float64 tensor of nx*ny*3")
            if not accum.is_cuda or accum.device.index != self.device:
                raise ValueError(f"a torch accum must live on this scene's GPU (cuda:{self.device})")
            torch.cuda.synchronize(accum.device)
            ptr = C.c_void_p(accum.data_ptr())
            on_device = 1
        prm = _abi.rtw_render_params(nx=nx, ny=ny, spp=spp, max_depth=max_depth, seed=seed, spp_begin=spp_begin,
                                     spp_count=spp_count, row_begin=row_begin, row_step=row_step,
                                     accum_on_device=on_device, collect_kernel_times=int(collect_kernel_times),
                                     wavefront_paths=wavefront_paths, precision=_precision(precision))
        st = _abi.rtw_stats()
        cam = camera if camera is not None else self.scene.camera
        check(lib().rtw_render_accumulate(self.handle, C.byref(cam), C.byref(prm), ptr, C.byref(st)),
              "rtw_render_accumulate")
        return accum, st.as_dict()

    def finalize_device(self, accum, nx: int, ny: int, spp: int, canvas=None):
        """canvas = min(sqrt(accum / spp), 1) on the GPU (torch float64 CUDA
        tensors of nx*ny*3 on this device).  Returns the canvas tensor."""
        import torch
        if not (accum.is_cuda and accum.dtype == torch.float64 and accum.numel() == nx * ny * 3
                and accum.is_contiguous()):
            raise ValueError("accum must be a contiguous float64 CUDA tensor of nx*ny*3")
        if canvas is None:
            canvas = torch.empty_like(accum)
        torch.cuda.synchronize(accum.device)
        check(lib().rtw_finalize_canvas_device(self.handle, C.c_void_p(accum.data_ptr()), nx, ny, spp,
                                               C.c_void_p(canvas.data_ptr())), "rtw_finalize_canvas_device")
        return canvas

    def query(self) -> dict:
        """rtw_scene_query: run layout, feature bits, the traversal kernel a
        render launches now and the device code's build id."""
        info = _abi.rtw_scene_info()
        check(lib().rtw_scene_query(self.handle, C.byref(info)), "rtw_scene_query")
        return info.as_dict()

    def quantize_device(self, canvas, nx: int, ny: int, out=None):
        """PPM channel values int(255.99f * c) of a device canvas, on the GPU
        (rtw_quantize_canvas_device).  Returns an int32 CUDA tensor."""
        import torch
        if not (canvas.is_cuda and canvas.dtype == torch.float64 and canvas.numel() == nx * ny * 3
                and canvas.is_contiguous()):
            raise ValueError("canvas must be a contiguous float64 CUDA tensor of nx*ny*3")
        if out is None:
            out = torch.empty(nx * ny * 3, dtype=torch.int32, device=canvas.device)
        torch.cuda.synchronize(canvas.device)
        check(lib().rtw_quantize_canvas_device(self.handle, C.c_void_p(canvas.data_ptr()), nx, ny,
                                               C.c_void_p(out.data_ptr())), "rtw_quantize_canvas_device")
        return out

    def close(self):
        if self.handle:
            lib().rtw_scene_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_multi(scenes, nx: int, ny: int, spp: int, max_depth: int, seed: int = 0, *, spp_begin: int = 0,
                 spp_count: int = 0, row_begin: int = 0, row_step: int = 1, accum=None,
                 camera: Optional[_abi.rtw_camera_desc] = None, collect_kernel_times: bool = False,
                 precision: str = "fp64"):
    """rtw_render_multi over DeviceScenes on distinct GPUs (one process, one
    host thread per GPU, RCCL reduce to scenes[0]'s device).  `accum`: float64
    numpy array, or torch float64 tensor on scenes[0]'s device."""
    if accum is None:
        accum = np.zeros(nx * ny * 3, dtype=np.float64)
    on_device = 0
    if isinstance(accum, np.ndarray):
        if accum.dtype != np.float64 or accum.size != nx * ny * 3 or not accum.flags["C_CONTIGUOUS"]:
            raise ValueError("accum must be a contiguous float64 array of nx*ny*3")
        ptr = accum.ctypes.data_as(C.c_void_p)
    else:
        import torch
        if accum.dtype != torch.float64 or accum.numel() != nx * ny * 3 or not accum.is_contiguous():
            raise ValueError("accum must be a contiguous float64 tensor of nx*ny*3")
        if not accum.is_cuda or accum.device.index != scenes[0].device:
            raise ValueError(f"a torch accum must live on scenes[0]'s GPU (cuda:{scenes[0].device})")
        torch.cuda.synchronize(accum.device)
        ptr = C.c_void_p(accum.data_ptr())
        on_device = 1
    handles = (C.c_void_p * len(scenes))(*[s.handle.value for s in scenes])
    prm = _abi.rtw_render_params(nx=nx, ny=ny, spp=spp, max_depth=max_depth, seed=seed, spp_begin=spp_begin,
                                 spp_count=spp_count, row_begin=row_begin, row_step=row_step,
                                 accum_on_device=on_device, collect_kernel_times=int(collect_kernel_times),
                                 wavefront_paths=0, precision=_precision(precision))
    st = _abi.rtw_stats()
    cam = camera if camera is not None else scenes[0].scene.camera
    check(lib().rtw_render_multi(len(scenes), handles, C.byref(cam), C.byref(prm), ptr, C.byref(st)),
          "rtw_render_multi")
    return accum, st.as_dict()


def _precision(name: str) -> int:
    try:
        return _abi.PRECISIONS[name]
    except KeyError:
        raise ValueError(f"precision must be one of {sorted(_abi.PRECISIONS)}, not {name!r}") from None


def write_ppm_quantized(path: str, rgb: np.ndarray, nx: int, ny: int) -> None:
    q = np.ascontiguousarray(rgb, dtype=np.int32)
    check(lib().rtw_write_ppm_quantized(str(path).encode(), q.ctypes.data_as(C.c_void_p), nx, ny),
          "rtw_write_ppm_quantized")


def build_id() -> str:
    return lib().rtw_build_id().decode()


def device_count() -> int:
    return lib().rtw_device_count()


def finalize(accum: np.ndarray, nx: int, ny: int, spp: int) -> np.ndarray:
    """canvas = min(sqrt(sum / spp), 1) (RayTracingWeekend.cpp:241-244), via the
    library's rtw_finalize_canvas."""
    a = np.ascontiguousarray(accum, dtype=np.float64)
    out = np.empty(nx * ny * 3, dtype=np.float64)
    lib().rtw_finalize_canvas(a.ctypes.data_as(C.c_void_p), nx, ny, spp, out.ctypes.data_as(C.c_void_p))
    return out


def write_ppm(path: str, canvas: np.ndarray, nx: int, ny: int) -> None:
    c = np.ascontiguousarray(canvas, dtype=np.float64)
    check(lib().rtw_write_ppm(str(path).encode(), c.ctypes.data_as(C.c_void_p), nx, ny), "rtw_write_ppm")


def render(scene: str, nx: int, ny: int, spp: int, max_depth: int, seed: int = 0, device: int = 0,
           use_bvh: bool = False, **kw) -> Tuple[np.ndarray, dict]:
    """Render `scene` at nx*ny*spp on one GPU; returns (canvas, stats)."""
    sd = SceneDesc(scene, nx * 1.0 / ny, use_bvh)
    ds = DeviceScene(sd, device)
    try:
        accum, stats = ds.render_accumulate(nx, ny, spp, max_depth, seed, **kw)
    finally:
        ds.close()
    return finalize(accum, nx, ny, spp), stats
