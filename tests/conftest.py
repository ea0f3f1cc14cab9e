import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def built():
    """The in-tree native library must exist: it is built beforehand on the
    CPU (`python -m raytracingweekend_amd.build`, the driver's build()), never
    inside a test -- a GPU session would otherwise spend its box time
    compiling.  A library older than its sources is reported, not rebuilt
    (measurements key on the library's own build id).  The oracle (gcc,
    seconds) is made if missing."""
    from raytracingweekend_amd import build
    if not build.LIB.exists():
        pytest.fail(f"{build.LIB} is missing: run `python -m raytracingweekend_amd.build` first")
    try:
        import ctypes
        lib = ctypes.CDLL(str(build.LIB))
        lib.rtw_build_id.restype = ctypes.c_char_p
        have, want = lib.rtw_build_id().decode(), build.build_id()
        if have != want:
            print(f"\nnote: {build.LIB.name} build id {have} != sources {want} (rebuild to test the sources)")
    except OSError:
        pass
    build.build_oracle()
    return True
