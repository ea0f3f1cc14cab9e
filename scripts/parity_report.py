"""Print the GPU-vs-oracle parity figures behind DESIGN.md: per case, the
max per-channel canvas difference, the PPM-byte mismatches and whether the
device-counted traversals equal the oracle's.  GPU box only (needs librtw.so
and the oracle build)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from oracle_lib import finalize_np, oracle_sums  # noqa: E402
from raytracingweekend_amd.render import DeviceScene, SceneDesc  # noqa: E402

CASES = [("cornell_box", 64, 64, 8, 50, False), ("cornell_box", 100, 100, 16, 50, False),
         ("random_balls", 120, 80, 8, 50, False), ("random_balls", 120, 80, 8, 50, True),
         ("dielectric", 96, 48, 16, 50, False), ("light_sample", 96, 48, 16, 50, False),
         ("book2_final", 48, 48, 4, 50, False), ("book2_final", 48, 48, 4, 50, True)]
for scene, nx, ny, spp, depth, bvh in CASES:
    ds = DeviceScene(SceneDesc(scene, nx / ny, use_bvh=bvh))
    acc, st = ds.render_accumulate(nx, ny, spp, depth, seed=7)
    ds.close()
    ref, seg = oracle_sums(SceneDesc(scene, nx / ny), nx, ny, spp, depth, seed=7)
    a, b = finalize_np(acc, spp), finalize_np(ref, spp)
    k = np.float64(np.float32(255.99))
    print(json.dumps({"scene": scene, "size": f"{nx}x{ny}x{spp}", "depth": depth, "bvh": bvh,
                      "max_abs_diff": float(np.abs(a - b).max()),
                      "ppm_byte_mismatches": int(((k * a).astype(np.int64) != (k * b).astype(np.int64)).sum()),
                      "channels": int(a.size), "segments_gpu": int(st["segments"]), "segments_oracle": int(seg)}),
          flush=True)
