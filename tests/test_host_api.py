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
    r = subprocess.run([str(cli), "--precision", "fp16"], capture_output=True, text=True)
    assert r.returncode == 2 and "expected fp64 or fp32" in r.stderr


def _minstd_canonical(n):
    """The first n values of libstdc++'s generate_canonical<double, 53> over a
    default-seeded std::minstd_rand (two raw draws per double)."""
    x, out = 1, []
    R = 2147483646.0
    for _ in range(n):
        x = x * 48271 % 2147483647
        e1 = float(x - 1)
        x = x * 48271 % 2147483647
        e2 = float(x - 1)
        r = (e1 + e2 * R) / float(R * R)
        out.append(r if r < 1.0 else 0.99999999999999989)
    return out


def test_reference_main_include_set_compiles_and_behaves(built, tmp_path):
    """A TU including every header RayTracingWeekend.cpp:20-30 names (vec3,
    onb, ray, pdf, sphere, hittable_list, camera, material, utility, scene)
    from this tree, exercising onb.h / pdf.h / utility.h and the light shapes'
    pdf_value / random (tests/cpp/test_ref_includes.cpp)."""
    exe = tmp_path / "test_ref_includes"
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", f"-I{ROOT / 'include'}", f"-I{PKG / 'csrc' / 'host'}",
           f"-I{PKG / 'csrc' / 'host' / 'rtw'}", str(ROOT / "tests" / "cpp" / "test_ref_includes.cpp"),
           f"-L{PKG}", "-lrtw", f"-Wl,-rpath,{PKG}", "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib",
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and "OK (0 failures)" in r.stdout, r.stdout + r.stderr
    vals = [float(x) for x in r.stdout.split("random_double ")[1].split()[:3]]
    u = _minstd_canonical(3)
    assert vals[0] == u[0] and vals[1] == u[1] and vals[2] == 2.0 + (4.0 - 2.0) * u[2]
