"""Host C++ scene API (CPU): the reference's CppTest assertions and a
reference-style user scene, compiled against raytracingweekend_amd's headers
and linked to librtw.so; plus the rtw_render host program's argument errors."""
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "raytracingweekend_amd"


def test_reference_style_scene_code_compiles_and_flattens(built, tmp_path):
    exe = tmp_path / "test_host_api"
    cmd = ["g++", "-std=c++17", "-O1", f"-I{ROOT / 'include'}", f"-I{PKG / 'csrc' / 'host'}",
           f"-I{PKG / 'csrc' / 'host' / 'rtw'}", str(ROOT / "tests" / "cpp" / "test_host_api.cpp"),
           f"-L{PKG}", "-lrtw", f"-Wl,-rpath,{PKG}", "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib",
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK (0 failures)" in r.stdout


def test_cli_rejects_unknown_scene(built):
    from raytracingweekend_amd import build
    cli = build.build_cli()
    r = subprocess.run([str(cli), "--scene", "nope"], capture_output=True, text=True)
    assert r.returncode == 2 and "unknown scene" in r.stderr
