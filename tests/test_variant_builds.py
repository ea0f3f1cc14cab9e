"""Every build variant the kernels keep behind a macro still compiles (CPU:
hipcc's gfx950 front end, -fsyntax-only over the one-kernel subset builds of
scripts/ru_kernel.sh, templates instantiated).  The variants are the A/B
forms measured and left off plus the strict-radiance
build; without this check a default-off path could rot unnoticed.
The default build is compiled in full by build() and run by the GPU suite;
the strict build likewise (tests/test_gpu_strict.py)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "raytracingweekend_amd" / "csrc"
HIPCC = "/opt/rocm/bin/hipcc"

T = ["-DRTW_SUBSET_F=112", "-DRTW_SUBSET_M=8", "-DRTW_SUBSET_L=true"]        # Cornell (T)
C3 = ["-DRTW_SUBSET_F=130", "-DRTW_SUBSET_M=12", "-DRTW_SUBSET_L=false"]    # random_balls + BVH
C5 = ["-DRTW_SUBSET_F=357", "-DRTW_SUBSET_M=29", "-DRTW_SUBSET_L=false"]    # Book-2 final + BVH
FAST5 = T + ["-DRTW_SUBSET_FAST", "-DRTW_SUBSET_FAST_F=5"]                  # fp32 Book-2 kernel

VARIANTS = {
    "strict_radiance": T + ["-DRTW_STRICT_RADIANCE=1"],
    "strict_radiance_media": C5 + ["-DRTW_STRICT_RADIANCE=1"],
    "canon_two_steps": T + ["-DRTW_CANON_ONESTEP=0"],
    "compiler_sqrt": T + ["-DRTW_SQRT_CORE=0"],
    "nt_records": T + ["-DRTW_NT_RECORDS=1"],
    "group_tos": C5 + ["-DRTW_GROUP_TOS=1"],
    "group_tos_fast": FAST5 + ["-DRTW_GROUP_TOS=1"],
    "no_rng_jump": T + ["-DRTW_RNG_JUMP=0", "-DRTW_PACKET_ALL=0"],
    "nt_records_fast": FAST5 + ["-DRTW_NT_RECORDS=1"],
    "sqrt_core_normalize": C5 + ["-DRTW_SQRT_NORM=1"],
    "sort_home_ray": T + ["-DRTW_SORT_HOME_RAY=1"],
    "div3_shared": T + ["-DRTW_DIV3_SHARED=1"],
    "pixel_major": T + ["-DRTW_PIXEL_MAJOR=1"],
    "key_order": T + ["-DRTW_KEY_ORDER=2"],
    "sort_mixture": T + ["-DRTW_SORT_MIXTURE=1"],
    "sort_prefix_plain": T + ["-DRTW_SORT_DPP=0"],
    "canon_min": T + ["-DRTW_CANON_MIN=1"],
    "seed_fold": T + ["-DRTW_SEED_FOLD=1"],
    "sqrt_unit_off": C3 + ["-DRTW_SQRT_UNIT=0"],
    "fast_lds_rangecheck": T + ["-DRTW_FAST_LDS_OFF=0"],
    "rect_early_return": T + ["-DRTW_RECT_BRANCHLESS=0"],
    "profiling": T + ["-DRTW_PROF"],
    "bvh4": C3 + ["-DRTW_BVH4=1"],
    "packet": C3 + ["-DRTW_PACKET=1"],
    "bin_rays": C3 + ["-DRTW_BIN_RAYS(F)=1"],
    "node16": C5 + ["-DRTW_NODE16=1"],
    "medium_cache": C5 + ["-DRTW_MEDIUM_CACHE=1"],
    "fuse_groups": C5 + ["-DRTW_FUSE_GROUPS=1"],
    "leaf_rcp": C5 + ["-DRTW_LEAF_RCP=1"],
    "persist_direct": C5 + ["-DRTW_PERSIST_DIRECT(F)=1"],
    "park_origin": C5 + ["-DRTW_PARK_ORIGIN(F)=1", "-DRTW_PBATCH(F)=32"],
    "fast_home": FAST5 + ["-DRTW_FAST_HOME(F)=1"],
}


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_variant_compiles(name):
    if not shutil.which(HIPCC) and not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    cmd = [HIPCC, "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
           f"-I{ROOT / 'include'}", f"-I{CSRC}", f"-I{CSRC / 'host'}", f"-I{CSRC / 'host' / 'rtw'}", "-DRTW_SUBSET",
           *VARIANTS[name], "-x", "hip", "--offload-device-only", "-fsyntax-only", str(CSRC / "rtw_kernels.hip")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
