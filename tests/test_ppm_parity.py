"""Whole-image P3 byte parity against the reference's own writer.

tests/golden/ppm_*.ppm were written by oracle/_ref/rtw_ref ppm (the
reference's classes, and RayTracingWeekend.cpp:235-276 -- average, gamma 2,
clamp, P3 rows ny-1..0, int(255.99f * c) -- restated in oracle/ref_harness.cpp
over the reference's own vec3); oracle/make_golden.py made them.

* CPU: the C restatement's sums -> this library's host finalize and writer
  (rtw_finalize_canvas, rtw_write_ppm) give the same bytes.
* GPU: the HIP render -> device finalize -> device quantize
  (rtw_quantize_canvas_device) -> rtw_write_ppm_quantized, and the host
  writer over the device canvas, give the same bytes.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest

from oracle_lib import oracle_sums

from raytracingweekend_amd.render import SceneDesc, finalize, write_ppm

GOLD = Path(__file__).resolve().parent / "golden"
CASES = json.loads((GOLD / "ppms.json").read_text())
IDS = [c["case"] for c in CASES]


def _aspect(c):
    return c["nx"] * 1.0 / c["ny"]  # RayTracingWeekend.cpp:204


@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_host_writer_matches_reference_ppm(c, tmp_path):
    sd = SceneDesc(c["scene"], _aspect(c))
    sums, _ = oracle_sums(sd, c["nx"], c["ny"], c["spp"], c["max_depth"], c["seed"])
    canvas = finalize(sums, c["nx"], c["ny"], c["spp"])
    out = tmp_path / "o.ppm"
    write_ppm(str(out), canvas, c["nx"], c["ny"])
    assert out.read_bytes() == (GOLD / f"ppm_{c['case']}.ppm").read_bytes()


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES, ids=IDS)
def test_gpu_image_matches_reference_ppm(c, tmp_path):
    import torch

    from raytracingweekend_amd.render import DeviceScene, write_ppm_quantized

    nx, ny, spp = c["nx"], c["ny"], c["spp"]
    sd = SceneDesc(c["scene"], _aspect(c))
    ds = DeviceScene(sd, 0)
    try:
        accum = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda:0")
        ds.render_accumulate(nx, ny, spp, c["max_depth"], c["seed"], accum=accum)
        canvas = ds.finalize_device(accum, nx, ny, spp)
        rgb = ds.quantize_device(canvas, nx, ny)
        torch.cuda.synchronize()
        a, b = tmp_path / "dev.ppm", tmp_path / "host.ppm"
        write_ppm_quantized(str(a), rgb.cpu().numpy(), nx, ny)
        write_ppm(str(b), canvas.cpu().numpy(), nx, ny)
    finally:
        ds.close()
    gold = (GOLD / f"ppm_{c['case']}.ppm").read_bytes()
    assert a.read_bytes() == gold, "device-quantized image differs from the reference's PPM"
    assert b.read_bytes() == gold, "host-written image of the device canvas differs from the reference's PPM"
