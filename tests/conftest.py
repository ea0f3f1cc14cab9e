import os
import sys
import warnings
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
    compiling.  A library older than its sources is reported (a warning in
    pytest's summary), not rebuilt -- measurements key on the library's own
    build id; RTW_REQUIRE_FRESH=1 makes it a failure.  The oracle (gcc,
    seconds) is made if missing."""
    from raytracingweekend_amd import _abi, build
    if not _abi.LIB_PATH.exists():
        pytest.fail(f"{_abi.LIB_PATH} is missing: run `python -m raytracingweekend_amd.build` first")
    # through _abi: torch's HIP runtime is loaded before the library's (the
    # other order breaks torch's GPU initialisation later in the session)
    have = _abi.lib().rtw_build_id().decode()
    if _abi.LIB_PATH == build.LIB:
        stale(build.LIB.name, have, build.build_id())
    build.build_oracle()
    return True


def stale(name: str, have: str, want: str) -> None:
    """A library whose build id is not the sources' (tests would judge another
    build): a warning, or a failure under RTW_REQUIRE_FRESH=1."""
    if have == want:
        return
    msg = f"{name} build id {have} != sources {want} (rebuild to test the sources)"
    if os.environ.get("RTW_REQUIRE_FRESH", "") == "1":
        pytest.fail(msg)
    warnings.warn(msg)
