"""Generate tests/golden/ from the reference's own code (oracle/_ref/rtw_ref,
built by oracle/Makefile from /root/reference) — TEST INFRASTRUCTURE ONLY.

Run in the dev container (where /root/reference exists):
    make -C oracle ref && python oracle/make_golden.py

Writes, for the parity tests (which must run where the reference is absent):
  scene_<name>.json      dump of the reference scene graph (every field)
  perlin.json            Perlin tables + noise/turb/texture known answers
  render_<case>.npy      per-pixel radiance sums (float64, nx*ny*3)
  renders.json           the cases: scene, size, spp, depth, seed, segments
  ppm_<case>.ppm         whole images as the reference writes them
                         (RayTracingWeekend.cpp:235-276: average, gamma 2,
                         clamp, P3 rows ny-1..0, int(255.99f * c))
  ppms.json              their cases
"""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
REF = ROOT / "oracle" / "_ref" / "rtw_ref"
OUT = ROOT / "tests" / "golden"

SCENES = [("cornell_box", 1.0), ("random_balls", 1.5), ("dielectric", 2.0), ("light_sample", 2.0),
          ("book2_final", 1.0), ("nested", 1.0), ("nested_plain", 1.0)]

# (case, scene, nx, ny, spp, depth, seed)
RENDERS = [
    ("cornell_32x32x4_d50", "cornell_box", 32, 32, 4, 50, 0),
    ("cornell_24x24x3_d100", "cornell_box", 24, 24, 3, 100, 5),
    ("cornell_20x20x2_d1", "cornell_box", 20, 20, 2, 1, 9),
    ("random_balls_48x32x4_d50", "random_balls", 48, 32, 4, 50, 0),
    ("random_balls_30x20x2_d100", "random_balls", 30, 20, 2, 100, 3),
    ("dielectric_32x16x4_d50", "dielectric", 32, 16, 4, 50, 0),
    ("light_sample_32x16x4_d50", "light_sample", 32, 16, 4, 50, 0),
    ("book2_final_16x16x2_d50", "book2_final", 16, 16, 2, 50, 0),
    ("nested_24x24x4_d50", "nested", 24, 24, 4, 50, 0),
    ("nested_32x24x3_d20", "nested", 32, 24, 3, 20, 3),
    ("nested_plain_24x24x4_d50", "nested_plain", 24, 24, 4, 50, 1),
]

# whole-image P3 files (case, scene, nx, ny, spp, depth, seed)
PPMS = [
    ("cornell_48x48x8_d50", "cornell_box", 48, 48, 8, 50, 0),
    ("random_balls_60x40x4_d50", "random_balls", 60, 40, 4, 50, 7),
]


def run(*args) -> str:
    r = subprocess.run([str(REF), *map(str, args)], check=True, capture_output=True, text=True)
    return r.stdout


def main() -> int:
    if not REF.exists():
        print(f"{REF} missing: run `make -C oracle ref` first (needs /root/reference)", file=sys.stderr)
        return 1
    OUT.mkdir(parents=True, exist_ok=True)
    for name, aspect in SCENES:
        dump = json.loads(run("scene", name, aspect))
        dump["aspect"] = aspect
        (OUT / f"scene_{name}.json").write_text(json.dumps(dump, separators=(",", ":")))
    (OUT / "perlin.json").write_text(json.dumps(json.loads(run("perlin")), separators=(",", ":")))
    meta = []
    for case, scene, nx, ny, spp, depth, seed in RENDERS:
        path = OUT / f"render_{case}.bin"
        info = json.loads(run("render", scene, nx, ny, spp, depth, seed, 8, path).strip().splitlines()[-1])
        sums = np.fromfile(path, dtype=np.float64)
        path.unlink()
        np.save(OUT / f"render_{case}.npy", sums)
        meta.append({"case": case, "scene": scene, "nx": nx, "ny": ny, "spp": spp, "max_depth": depth,
                     "seed": seed, "segments": info["segments"]})
    (OUT / "renders.json").write_text(json.dumps(meta, indent=1))
    ppm_meta = []
    for case, scene, nx, ny, spp, depth, seed in PPMS:
        run("ppm", scene, nx, ny, spp, depth, seed, 8, OUT / f"ppm_{case}.ppm")
        ppm_meta.append({"case": case, "scene": scene, "nx": nx, "ny": ny, "spp": spp, "max_depth": depth,
                         "seed": seed})
    (OUT / "ppms.json").write_text(json.dumps(ppm_meta, indent=1))
    print(f"wrote {len(SCENES)} scenes, perlin, {len(RENDERS)} renders, {len(PPMS)} ppm images to {OUT}")
    return 0


# ---------------------------------------------------------------------------
# Statistical fixture: the reference's committed render of its default
# configuration (Sampling/glassball.png: cornell_box 400x400, 64 spp, depth 100,
# rendered by the reference with its shared global RNG).  Stored as statistics
# only (channel means and 16x16-block means of the 8-bit image).
# ---------------------------------------------------------------------------
def decode_png_rgb8(path: Path) -> np.ndarray:
    import struct
    import zlib
    d = path.read_bytes()
    assert d[:8] == b"\x89PNG\r\n\x1a\n"
    i, idat = 8, b""
    w = h = None
    while i < len(d):
        n, = struct.unpack(">I", d[i:i + 4])
        t = d[i + 4:i + 8]
        body = d[i + 8:i + 8 + n]
        if t == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert depth == 8 and ctype == 2, "expects 8-bit RGB"
        elif t == b"IDAT":
            idat += body
        i += 12 + n
    raw = zlib.decompress(idat)
    bpp, stride = 3, w * 3
    img = np.zeros((h, stride), dtype=np.int64)
    prev = np.zeros(stride, dtype=np.int64)
    pos = 0
    for y in range(h):
        f = raw[pos]
        line = np.frombuffer(raw[pos + 1:pos + 1 + stride], dtype=np.uint8).astype(np.int64)
        pos += 1 + stride
        out = np.zeros(stride, dtype=np.int64)
        for x in range(stride):
            a = out[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            if f == 0:
                p = 0
            elif f == 1:
                p = a
            elif f == 2:
                p = b
            elif f == 3:
                p = (a + b) // 2
            else:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            out[x] = (line[x] + p) & 255
        img[y] = out
        prev = out
    return img.reshape(h, w, 3)


def glassball_stats():
    png = Path("/root/reference/RayTracingWeekend/Sampling/glassball.png")
    img = decode_png_rgb8(png).astype(np.float64)  # row 0 = top of the image
    blocks = img.reshape(25, 16, 25, 16, 3).mean(axis=(1, 3))
    return {"source": "RayTracingWeekend/Sampling/glassball.png", "config": {
        "scene": "cornell_box", "nx": 400, "ny": 400, "spp": 64, "max_depth": 100},
        "channel_mean": img.mean(axis=(0, 1)).tolist(), "block16_mean": blocks.tolist()}


if __name__ == "__main__":
    rc = main()
    if rc == 0:
        (OUT / "glassball_stats.json").write_text(json.dumps(glassball_stats()))
    sys.exit(rc)
