"""The C-ABI library (CPU): it loads, exports every function include/rtw_gpu.h
declares, its struct layouts agree with the ctypes mirror, host-side entry
points behave (PPM bytes, finalize, error reporting).  No GPU compute here."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from raytracingweekend_amd import _abi

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "rtw_gpu.h"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(rtw_[a-z_0-9]+)\s*\(", text)))


def test_every_declared_symbol_is_exported(built):
    lib = _abi.lib()
    names = declared_functions()
    assert len(names) == 18
    for n in names:
        assert hasattr(lib, n), f"{n} declared in rtw_gpu.h but not exported"
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_abi.LIB_PATH)], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}$", nm, re.M), f"{n} is not a defined text symbol"
    assert set(names) == set(_abi.SIGNATURES)


STRUCTS = ["rtw_prim", "rtw_entry", "rtw_bvh_node", "rtw_material", "rtw_texture", "rtw_light", "rtw_camera_desc",
           "rtw_scene_desc", "rtw_render_params", "rtw_stats", "rtw_scene_info"]


def test_struct_layouts_match_c(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rtw_gpu.h"', "int main(void){"]
    for s in STRUCTS:
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f, _ in getattr(_abi, s)._fields_:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.split("\n") if l)
    for s in STRUCTS:
        cls = getattr(_abi, s)
        assert int(out[s]) == C.sizeof(cls), s
        for f, _ in cls._fields_:
            assert int(out[f"{s}.{f}"]) == getattr(cls, f).offset, f"{s}.{f}"
    # sizes documented in the header
    assert C.sizeof(_abi.rtw_prim) == 96 and C.sizeof(_abi.rtw_entry) == 312
    assert C.sizeof(_abi.rtw_bvh_node) == 64 and C.sizeof(_abi.rtw_material) == 48


def test_ppm_writer_bytes(built, tmp_path):
    """RayTracingWeekend.cpp:257-276: header, rows top to bottom, int(255.99f*c)."""
    from raytracingweekend_amd.render import write_ppm
    nx, ny = 3, 2
    canvas = np.zeros((ny, nx, 3))
    canvas[0, 0] = [1.0, 0.5, 0.0]        # bottom-left pixel (j = 0)
    canvas[1, 2] = [0.999, 0.25, 0.0039]  # top-right pixel (j = 1)
    p = tmp_path / "x.ppm"
    write_ppm(str(p), canvas.reshape(-1), nx, ny)
    k = float(np.float32(255.99))
    q = lambda v: int(k * v)  # noqa: E731
    want = "P3\n3 2\n255\n" + "0 0 0\n0 0 0\n" + f"{q(0.999)} {q(0.25)} {q(0.0039)}\n" + \
           f"{q(1.0)} {q(0.5)} 0\n0 0 0\n0 0 0\n"
    assert p.read_text() == want
    assert q(1.0) == 255 and q(0.5) == 127


def test_error_reporting_without_device(built):
    lib = _abi.lib()
    from raytracingweekend_amd.render import SceneDesc
    sd = SceneDesc("cornell_box", 1.0)
    bad = _abi.rtw_scene_desc.from_buffer_copy(sd.desc)
    bad.abi_version = 99
    h = C.c_void_p()
    rc = lib.rtw_scene_upload(0, C.byref(bad), C.byref(h))
    assert rc == -1 and b"ABI" in lib.rtw_last_error()
    bad = _abi.rtw_scene_desc.from_buffer_copy(sd.desc)
    bad.n_prims = 3  # entries now reference prims out of range
    assert lib.rtw_scene_upload(0, C.byref(bad), C.byref(h)) == -1
    assert b"out of bounds" in lib.rtw_last_error()
    if lib.rtw_device_count() == 0:
        rc = lib.rtw_scene_upload(0, sd.ptr, C.byref(h))
        assert rc == -3 and h.value is None
    assert lib.rtw_render_accumulate(None, None, None, None, None) == -1


def _bad_owner_desc(sd, mutate):
    """A copy of sd's desc whose prim array is a private copy changed by
    `mutate(prims)` (the library-owned arrays stay untouched)."""
    d = _abi.rtw_scene_desc.from_buffer_copy(sd.desc)
    prims = (_abi.rtw_prim * d.n_prims)()
    C.memmove(prims, d.prims, C.sizeof(prims))
    mutate(prims)
    d.prims = C.cast(prims, C.POINTER(_abi.rtw_prim))
    return d, prims


def test_upload_rejects_prims_their_entries_do_not_own(built):
    """validate_desc's ownership rule (rtw_kernels.hip validate_desc): every
    prim of an entry's range names that entry, and a light's own copy names
    none -- hit_record reads the winner's transforms through prims[i].entry,
    so a desc breaking it would index entries out of their range."""
    lib = _abi.lib()
    from raytracingweekend_amd.render import SceneDesc
    sd = SceneDesc("cornell_box", 1.0)
    h = C.c_void_p()
    e0 = sd.desc.entries[0]
    # a prim inside entry 0's range naming entry 1
    d, keep = _bad_owner_desc(sd, lambda P: setattr(P[e0.first_prim], "entry", 1))
    assert lib.rtw_scene_upload(0, C.byref(d), C.byref(h)) == -1
    assert b"lies in entry" in lib.rtw_last_error() and h.value is None
    # a light's own copy (outside every range) claiming an entry
    n = sd.desc.n_prims
    d, keep = _bad_owner_desc(sd, lambda P: setattr(P[n - 1], "entry", 0))
    assert lib.rtw_scene_upload(0, C.byref(d), C.byref(h)) == -1
    assert b"names entry" in lib.rtw_last_error()
    # an entry index past the end
    d, keep = _bad_owner_desc(sd, lambda P: setattr(P[0], "entry", sd.desc.n_entries))
    assert lib.rtw_scene_upload(0, C.byref(d), C.byref(h)) == -1
    assert b"entry out of range" in lib.rtw_last_error()
    # two entries claiming one prim
    bad = _abi.rtw_scene_desc.from_buffer_copy(sd.desc)
    ents = (_abi.rtw_entry * bad.n_entries)()
    C.memmove(ents, bad.entries, C.sizeof(ents))
    ents[1].first_prim = ents[0].first_prim
    ents[1].n_prims = 1
    bad.entries = C.cast(ents, C.POINTER(_abi.rtw_entry))
    assert lib.rtw_scene_upload(0, C.byref(bad), C.byref(h)) == -1
    assert b"belongs to entries" in lib.rtw_last_error()


def test_render_multi_argument_errors(built):
    """rtw_render_multi refuses bad arguments before touching any device."""
    lib = _abi.lib()
    from raytracingweekend_amd.render import SceneDesc
    sd = SceneDesc("cornell_box", 1.0)
    prm = _abi.rtw_render_params(nx=8, ny=8, spp=1, max_depth=5, row_step=1)
    acc = np.zeros(8 * 8 * 3)
    hs = (C.c_void_p * 2)(None, None)
    for n in (0, -1):
        assert lib.rtw_render_multi(n, hs, C.byref(sd.camera), C.byref(prm), acc.ctypes.data_as(C.c_void_p),
                                    None) == -1
    assert lib.rtw_render_multi(2, hs, C.byref(sd.camera), C.byref(prm), acc.ctypes.data_as(C.c_void_p),
                                None) == -1
    assert b"null scene handle" in lib.rtw_last_error()
    assert lib.rtw_render_multi(1, None, C.byref(sd.camera), C.byref(prm), acc.ctypes.data_as(C.c_void_p),
                                None) == -1


def test_precision_names():
    from raytracingweekend_amd.render import _precision
    assert _precision("fp64") == _abi.RTW_PRECISION_FP64 == 0
    assert _precision("fp32") == _abi.RTW_PRECISION_FP32 == 1
    with pytest.raises(ValueError):
        _precision("bf16")


def test_library_refuses_to_fall_back(tmp_path):
    """A missing librtw.so is an error, never a silent CPU path."""
    import os
    import sys
    env = dict(os.environ, RTW_LIBRARY=str(tmp_path / "missing.so"), PYTHONPATH=str(ROOT))
    code = "from raytracingweekend_amd import render; render.SceneDesc('cornell_box', 1.0)"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    assert r.returncode != 0 and "no CPU fallback" in r.stderr
