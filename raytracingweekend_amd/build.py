"""Build the native pieces in-tree (no JIT cache: the .so files travel to the
GPU box with the repository snapshot).

  raytracingweekend_amd/librtw.so     HIP kernels (gfx950) + C ABI + host scene API
  raytracingweekend_amd/_build/librtw_strict.so
                                      the strict-radiance build (RTW_STRICT_RADIANCE)
  raytracingweekend_amd/rtw_render    C++ host program (the reference's main())
  oracle/_ref/librtw_oracle.so        test-only C restatement (oracle/Makefile)
  oracle/_ref/rtw_ref                 test-only reference harness, only where
                                      /root/reference exists

Run:  python -m raytracingweekend_amd.build [--force]
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "_build"
LIB = PKG / "librtw.so"
CLI = PKG / "rtw_render"
ARCH = os.environ.get("RTW_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

INCLUDES = [f"-I{ROOT / 'include'}", f"-I{CSRC}", f"-I{CSRC / 'host'}", f"-I{CSRC / 'host' / 'rtw'}"]
# -ffp-contract=off: the reference's fp64 arithmetic is unfused (x86-64 g++
# emits no FMA), parity needs the same roundings on the device.
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-variable",
          "-Wno-unused-but-set-variable"]
# -fno-slp-vectorize: the SLP vectorizer folds chains of fp64 compares (the
# rect bounds tests) into i1-vector reductions that gfx950 evaluates lane by
# lane with cndmask / shift / bitop3 (19 VALU instead of 8 per rect test).
DEVICE = [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-fno-slp-vectorize"]

HOST_SOURCES = sorted((CSRC / "host").glob("*.cpp"))
DEVICE_SOURCES = sorted(CSRC.glob("*.hip"))
HEADERS = sorted(list(CSRC.rglob("*.h")) + [ROOT / "include" / "rtw_gpu.h"])
# what the device sources include: the build id and the kernels' rebuilds
# follow these only (the host scene API headers under csrc/host/rtw/ do not
# reach the kernels)
DEVICE_HEADERS = sorted([*CSRC.glob("rtw_*.h"), CSRC / "host" / "rtw_host_util.h", ROOT / "include" / "rtw_gpu.h"])
# RCCL for rtw_render_multi (multi.cpp); the same librccl.so.1 torch loads
LIBS = ["-L/opt/rocm/lib", "-lrccl"]


def build_id(extra=()) -> str:
    """Hash of the device code: kernel sources, headers and compile flags
    (compiled in as RTW_BUILD_ID; bench.py matches PMC files against it)."""
    h = hashlib.sha1()
    for f in [*DEVICE_SOURCES, *DEVICE_HEADERS]:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    h.update(" ".join([*DEVICE, *COMMON, *extra]).encode())
    return h.hexdigest()[:16]


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def _link(objs, out: Path) -> None:
    """Link into a temporary file and rename it over `out` (atomic: a
    snapshot of the tree taken meanwhile sees the old library or the new
    one, never a half-written file)."""
    tmp = out.with_name(out.name + ".tmp")
    _run([HIPCC, *DEVICE, "-shared", "-fPIC", *map(str, objs), *LIBS, "-o", str(tmp)])
    os.replace(tmp, out)


def _compile(src: Path, force: bool, extra=(), tag: str = "") -> Path:
    obj = BUILD / (src.name + tag + ".o")
    deps = DEVICE_HEADERS if src.suffix == ".hip" else HEADERS
    if force or _newer(obj, [src, *deps, Path(__file__)]):
        if src.suffix == ".hip":
            bid = f'-DRTW_BUILD_ID="{build_id(extra)}"'
            cmd = [HIPCC, *DEVICE, *COMMON, *extra, bid, *INCLUDES, "-x", "hip", "-c", str(src), "-o", str(obj)]
        else:
            cmd = [HIPCC, *COMMON, *extra, *INCLUDES, "-c", str(src), "-o", str(obj)]
        _run(cmd)
    return obj


def build_library(force: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    srcs = DEVICE_SOURCES + HOST_SOURCES
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or _newer(LIB, objs):
        _link(objs, LIB)
    return LIB


def build_variant_library(name: str, defines, force: bool = False, host: bool = False) -> Path:
    """_build/librtw_<name>.so: the library with extra -D flags on the kernels
    (and, host=True, on the host sources too: defines that change shared
    layouts); tuning experiments, select with RTW_LIBRARY=..."""
    BUILD.mkdir(exist_ok=True)
    out = BUILD / f"librtw_{name}.so"
    flags = [f"-D{d}" for d in defines]
    objs = [_compile(s, force, flags, f".{name}") for s in DEVICE_SOURCES]
    objs += [_compile(s, force, flags, f".{name}") if host else _compile(s, force) for s in HOST_SOURCES]
    if force or _newer(out, objs):
        _link(objs, out)
    return out


def build_profiling_library(force: bool = False) -> Path:
    """_build/librtw_prof.so: the same library with the kernels' section
    profiler compiled in (-DRTW_PROF); select it with RTW_LIBRARY=... .
    A measurement tool only: its timers perturb the kernels."""
    BUILD.mkdir(exist_ok=True)
    out = BUILD / "librtw_prof.so"
    objs = [_compile(s, force, ["-DRTW_PROF"], ".prof") for s in DEVICE_SOURCES]
    objs += [_compile(s, force) for s in HOST_SOURCES]
    if force or _newer(out, objs):
        _link(objs, out)
    return out


def build_cli(force: bool = False) -> Path:
    src = CSRC / "tools" / "rtw_render.cpp"
    if src.exists() and (force or _newer(CLI, [src, LIB, *HEADERS])):
        _run([HIPCC, *COMMON, *INCLUDES, str(src), f"-L{PKG}", "-lrtw", f"-Wl,-rpath,$ORIGIN", "-o", str(CLI)])
    return CLI


def build_oracle(force: bool = False) -> None:
    """Test-only checker (oracle/): the C restatement always; the reference
    harness only where the reference sources exist (this container)."""
    targets = ["port"]
    if Path(os.environ.get("RTW_REFERENCE_DIR", "/root/reference/RayTracingWeekend")).is_dir():
        targets.append("ref")
    if force:
        _run(["make", "-C", str(ROOT / "oracle"), "-B", *targets])
    else:
        _run(["make", "-C", str(ROOT / "oracle"), *targets])


def build_test_tools(force: bool = False) -> None:
    """Test-only HIP programs (tests/cpp/*.hip) -> _build/<name>: checks that
    run on the card (tests/test_div_hw.py)."""
    BUILD.mkdir(exist_ok=True)
    for src in sorted((ROOT / "tests" / "cpp").glob("*.hip")):
        out = BUILD / src.stem
        if force or _newer(out, [src, *HEADERS]):
            _run([HIPCC, *DEVICE, *COMMON, *INCLUDES, "-x", "hip", str(src), "-o", str(out)])


STRICT_LIB = BUILD / "librtw_strict.so"


def build_strict_library(force: bool = False) -> Path:
    """_build/librtw_strict.so: the strict-radiance build (RTW_STRICT_RADIANCE:
    the reference's radiance arithmetic, each path's factors folded
    inside-out as color() returns them), checked to the last bit against the
    oracle's device-libm build by tests/test_gpu_strict.py."""
    # (host=True: its own host objects too, so a concurrent build_library
    # never compiles into the same object file)
    out = build_variant_library("strict", ["RTW_STRICT_RADIANCE=1"], force, host=True)
    assert out == STRICT_LIB
    return out


def build_all(force: bool = False) -> None:
    # the product library and the strict-radiance build compile their
    # kernels concurrently (one translation unit each)
    with ThreadPoolExecutor(max_workers=2) as ex:
        jobs = [ex.submit(build_library, force), ex.submit(build_strict_library, force)]
        for j in jobs:
            j.result()
    build_cli(force)
    build_oracle(force)
    build_test_tools(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print(f"built {LIB}")
