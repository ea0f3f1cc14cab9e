"""ctypes mirror of include/rtw_gpu.h (field for field) and the library loader.

The library is the in-tree librtw.so built by raytracingweekend_amd.build; a
missing library is an error, never a silent fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("RTW_LIBRARY", PKG / "librtw.so"))

RTW_ABI_VERSION = 3
RTW_MAX_OPS = 8

# enums (rtw_gpu.h)
RTW_PRIM_SPHERE, RTW_PRIM_MOVING_SPHERE, RTW_PRIM_RECT_XY, RTW_PRIM_RECT_XZ, RTW_PRIM_RECT_YZ = range(5)
RTW_OP_TRANSLATE, RTW_OP_ROTATE_Y, RTW_OP_FLIP = 1, 2, 3
RTW_ENTRY_GROUP, RTW_ENTRY_MEDIUM = 0, 1
RTW_MAT_LAMBERTIAN, RTW_MAT_METAL, RTW_MAT_DIELECTRIC, RTW_MAT_DIFFUSE_LIGHT, RTW_MAT_ISOTROPIC = range(5)
RTW_TEX_CONSTANT, RTW_TEX_CHECKER, RTW_TEX_NOISE = range(3)
RTW_LIGHT_DEFAULT, RTW_LIGHT_XZ_RECT, RTW_LIGHT_SPHERE = range(3)
RTW_RENDER_SHADED, RTW_RENDER_NORMAL = 0, 1
RTW_BG_BLACK, RTW_BG_GRADIENT = 0, 1
RTW_PRECISION_FP64, RTW_PRECISION_FP32 = 0, 1
RTW_ITEM_BOX, RTW_ITEM_INDEX = 0x40000000, 0x3FFFFFFF
RTW_VISIT_REPLAY, RTW_VISIT_ENTRY = 0x40000000, 0x3FFFFFFF
PRECISIONS = {"fp64": RTW_PRECISION_FP64, "fp32": RTW_PRECISION_FP32}


class rtw_prim(C.Structure):
    _fields_ = [("type", C.c_int32), ("material", C.c_int32), ("flip", C.c_int32), ("entry", C.c_int32),
                ("p", C.c_double * 10)]


class rtw_entry(C.Structure):
    _fields_ = [("kind", C.c_int32), ("first_prim", C.c_int32), ("n_prims", C.c_int32), ("n_ops", C.c_int32),
                ("op", C.c_int32 * RTW_MAX_OPS), ("phase_material", C.c_int32), ("bvh_root", C.c_int32),
                ("n_outer_ops", C.c_int32), ("pad", C.c_int32),
                ("op_param", (C.c_double * 3) * RTW_MAX_OPS), ("density", C.c_double), ("bounds", C.c_double * 6)]


class rtw_bvh_node(C.Structure):
    _fields_ = [("bmin", C.c_double * 3), ("bmax", C.c_double * 3), ("left", C.c_int32), ("right", C.c_int32),
                ("count", C.c_int32), ("pad", C.c_int32)]


class rtw_material(C.Structure):
    _fields_ = [("type", C.c_int32), ("texture", C.c_int32), ("albedo", C.c_double * 3), ("fuzz", C.c_double),
                ("ref_idx", C.c_double)]


class rtw_texture(C.Structure):
    _fields_ = [("type", C.c_int32), ("odd", C.c_int32), ("even", C.c_int32), ("pad", C.c_int32),
                ("color", C.c_double * 3), ("scale", C.c_double)]


class rtw_light(C.Structure):
    _fields_ = [("kind", C.c_int32), ("prim", C.c_int32)]


class rtw_camera_desc(C.Structure):
    _fields_ = [("origin", C.c_double * 3), ("lower_left", C.c_double * 3), ("horizontal", C.c_double * 3),
                ("vertical", C.c_double * 3), ("u", C.c_double * 3), ("v", C.c_double * 3), ("w", C.c_double * 3),
                ("time0", C.c_double), ("time1", C.c_double), ("lens_radius", C.c_double)]


class rtw_scene_desc(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("render_type", C.c_int32), ("background", C.c_int32),
                ("n_prims", C.c_int32), ("n_entries", C.c_int32), ("n_materials", C.c_int32),
                ("n_textures", C.c_int32), ("n_lights", C.c_int32), ("n_bvh_nodes", C.c_int32),
                ("n_bvh_items", C.c_int32), ("world_bvh_root", C.c_int32), ("has_perlin", C.c_int32),
                ("prims", C.POINTER(rtw_prim)), ("entries", C.POINTER(rtw_entry)),
                ("materials", C.POINTER(rtw_material)), ("textures", C.POINTER(rtw_texture)),
                ("lights", C.POINTER(rtw_light)), ("bvh_nodes", C.POINTER(rtw_bvh_node)),
                ("bvh_items", C.POINTER(C.c_int32)), ("perlin_ranvec", C.POINTER(C.c_double)),
                ("perlin_perm", C.POINTER(C.c_int32)), ("camera", rtw_camera_desc),
                ("visits", C.POINTER(C.c_int32)), ("n_visits", C.c_int32), ("pad", C.c_int32)]


class rtw_render_params(C.Structure):
    _fields_ = [("nx", C.c_int32), ("ny", C.c_int32), ("spp", C.c_int32), ("max_depth", C.c_int32),
                ("seed", C.c_uint64), ("spp_begin", C.c_int32), ("spp_count", C.c_int32),
                ("row_begin", C.c_int32), ("row_step", C.c_int32), ("accum_on_device", C.c_int32),
                ("collect_kernel_times", C.c_int32), ("wavefront_paths", C.c_int32), ("precision", C.c_int32)]


class rtw_stats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("segments", C.c_uint64), ("iterations", C.c_uint64),
                ("launches_intersect", C.c_uint64), ("ms_total", C.c_double), ("ms_intersect", C.c_double),
                ("ms_shade", C.c_double), ("ms_finalize", C.c_double), ("bytes_intersect", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class rtw_scene_info(C.Structure):
    _fields_ = [("device", C.c_int32), ("n_world_runs", C.c_int32), ("n_ysphere_runs", C.c_int32),
                ("n_plain_runs", C.c_int32), ("features", C.c_int32), ("shade_mask", C.c_int32),
                ("shade_lds_bytes", C.c_int32), ("bvh_lds_nodes", C.c_int32), ("kernel", C.c_char * 128),
                ("build_id", C.c_char * 48), ("kernel_fast", C.c_char * 128)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        for k in ("kernel", "build_id", "kernel_fast"):
            d[k] = d[k].decode()
        return d


# exported symbols and their signatures (the C ABI of include/rtw_gpu.h)
SIGNATURES = {
    "rtw_device_count": (C.c_int, []),
    "rtw_scene_upload": (C.c_int, [C.c_int, C.POINTER(rtw_scene_desc), C.POINTER(C.c_void_p)]),
    "rtw_render_accumulate": (C.c_int, [C.c_void_p, C.POINTER(rtw_camera_desc), C.POINTER(rtw_render_params),
                                        C.c_void_p, C.POINTER(rtw_stats)]),
    "rtw_finalize_canvas": (None, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "rtw_write_ppm": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
    "rtw_finalize_canvas_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "rtw_scene_free": (None, [C.c_void_p]),
    "rtw_last_error": (C.c_char_p, []),
    "rtw_path_seed": (C.c_uint32, [C.c_uint64, C.c_uint32, C.c_uint32]),
    "rtw_scene_builtin": (C.c_int, [C.c_char_p, C.c_double, C.c_int, C.POINTER(C.POINTER(rtw_scene_desc))]),
    "rtw_scene_desc_free": (None, [C.POINTER(rtw_scene_desc)]),
    "rtw_abi_version": (C.c_int, []),
    "rtw_render_multi": (C.c_int, [C.c_int, C.POINTER(C.c_void_p), C.POINTER(rtw_camera_desc),
                                   C.POINTER(rtw_render_params), C.c_void_p, C.POINTER(rtw_stats)]),
    "rtw_release_communicators": (None, []),
    "rtw_scene_query": (C.c_int, [C.c_void_p, C.POINTER(rtw_scene_info)]),
    "rtw_build_id": (C.c_char_p, []),
    "rtw_quantize_canvas_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "rtw_write_ppm_quantized": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
}

_lib = None


def load_library(path) -> C.CDLL:
    """Load a build of the library (librtw.so, or a variant such as
    _build/librtw_strict.so) with the C ABI's signatures.  Raises if it is
    missing: there is no CPU fallback."""
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7
    # (same soname as /opt/rocm's), and torch's GPU init fails if the
    # system runtime was loaded first -- so let torch load it first.
    if os.environ.get("RTW_NO_TORCH") != "1" and "torch" not in sys.modules:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    path = Path(path)
    if not path.exists():
        raise RuntimeError(f"native library {path} is missing: build it with "
                           f"`python -m raytracingweekend_amd.build` (there is no CPU fallback)")
    L = C.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.rtw_abi_version() != RTW_ABI_VERSION:
        raise RuntimeError(f"{path.name} ABI version mismatch; rebuild")
    return L


def lib():
    """Load librtw.so (once).  Raises if the native library is missing."""
    global _lib
    if _lib is None:
        _lib = load_library(LIB_PATH)
    return _lib


class RtwError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().rtw_last_error()
        raise RtwError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
