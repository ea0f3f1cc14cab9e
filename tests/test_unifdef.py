"""scripts/unifdef.py, the tool that pruned the rejected kernel variants in
round 6 (EXPERIMENTS.md): conditionals whose value the given macros fix are
resolved (their lines and the branches not taken dropped), every other
conditional is kept as written, with known-false #elif branches dropped and a
known-true #elif turned into the chain's #else."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

SRC = """a
#ifndef RTW_X
#define RTW_X 0
#endif
#if RTW_X
x1
#elif defined(FOO)
foo
#else
notx
#endif
#if FOO
#if RTW_Y && RTW_X
no
#else
yes
#endif
#elif RTW_Y
ybranch
#elif BAR
bar
#else
z
#endif
#if RTW_Y
#if BAZ
b
#endif
#endif
"""

WANT = """a
#if defined(FOO)
foo
#else
notx
#endif
#if FOO
yes
#else
ybranch
#endif
#if BAZ
b
#endif
"""


def test_unifdef_resolves_known_macros_only(tmp_path):
    f = tmp_path / "t.h"
    f.write_text(SRC)
    r = subprocess.run([sys.executable, str(ROOT / "scripts" / "unifdef.py"), "-DRTW_X=0", "-DRTW_Y=1", str(f)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert f.read_text() == WANT


def test_unifdef_leaves_unknown_conditionals(tmp_path):
    f = tmp_path / "u.h"
    f.write_text(SRC)
    subprocess.run([sys.executable, str(ROOT / "scripts" / "unifdef.py"), "-DOTHER=1", str(f)], check=True)
    assert f.read_text() == SRC
