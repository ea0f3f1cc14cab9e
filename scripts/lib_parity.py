"""Bit-identity of a variant library against the in-tree one (GPU box).

    python scripts/lib_parity.py [--fp32] <variant.so> [scene ...]

Renders each scene (small image) once per library, each in its own process
(the library is chosen at import by RTW_LIBRARY), and compares the
accumulated sums bit for bit.  Exit status 1 on any difference."""
import os
import subprocess
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = {"cornell_box": (96, 96, 64, False), "book2_final": (64, 64, 16, True),
         "random_balls": (96, 64, 16, True), "light_sample": (64, 64, 32, False),
         "random_balls_flat": (96, 64, 16, False)}


def _one(scene, out, precision):
    from raytracingweekend_amd.render import DeviceScene, SceneDesc
    nx, ny, spp, bvh = CASES[scene]
    ds = DeviceScene(SceneDesc(scene.replace("_flat", ""), nx / ny, bvh), 0)
    try:
        accum, _ = ds.render_accumulate(nx, ny, spp, 50, 7, precision=precision)
    finally:
        ds.close()
    np.save(out, np.asarray(accum))


def main():
    if sys.argv[1] == "--one":
        _one(sys.argv[2], sys.argv[3], sys.argv[4])
        return 0
    args = sys.argv[1:]
    precision = "fp64"
    if args[0] == "--fp32":
        precision, args = "fp32", args[1:]
    variant, scenes = args[0], args[1:] or sorted(CASES)
    bad = 0
    with tempfile.TemporaryDirectory() as d:
        for s in scenes:
            outs = []
            for lib in (None, variant):
                env = dict(os.environ)
                env.pop("RTW_LIBRARY", None)
                if lib:
                    env["RTW_LIBRARY"] = lib
                out = os.path.join(d, f"{s}_{len(outs)}.npy")
                subprocess.run([sys.executable, __file__, "--one", s, out, precision], env=env, check=True, timeout=300)
                outs.append(np.load(out))
            same = np.array_equal(outs[0].view(np.uint64), outs[1].view(np.uint64))
            print(f"{s} {precision}: {'identical' if same else 'DIFFERS (max abs %g)' % np.abs(outs[0] - outs[1]).max()}")
            bad += not same
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
