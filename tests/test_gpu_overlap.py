"""Overlapped passes (RTW_OVERLAP = n: the render split into n passes on two
streams, each pass's ordered reduction on a third stream while the next pass
traces) leave every pixel's sum bit for bit what one pass gives: the records
are reduced pass after pass into the running sums, so each pixel still adds
its samples in sample order (RayTracingWeekend.cpp:235-239).  Traversal
counts are unchanged too (the per-pass counters are summed)."""
import os

import numpy as np
import pytest

CASES = [("cornell_box", 64, 48, 64, False, "fp64"), ("random_balls", 48, 32, 24, True, "fp64"),
         ("book2_final", 32, 32, 16, True, "fp64"), ("cornell_box", 64, 48, 64, False, "fp32"),
         ("book2_final", 32, 32, 16, True, "fp32")]


def _render(scene, nx, ny, spp, bvh, precision, overlap):
    from raytracingweekend_amd.render import DeviceScene, SceneDesc
    old = os.environ.get("RTW_OVERLAP")
    os.environ["RTW_OVERLAP"] = str(overlap)
    try:
        ds = DeviceScene(SceneDesc(scene, nx / ny, bvh), 0)
        try:
            acc, st = ds.render_accumulate(nx, ny, spp, 50, 3, precision=precision)
        finally:
            ds.close()
    finally:
        if old is None:
            os.environ.pop("RTW_OVERLAP", None)
        else:
            os.environ["RTW_OVERLAP"] = old
    return np.asarray(acc), st


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[5]}" for c in CASES])
def test_overlapped_passes_are_bit_identical(built, case):
    one, st1 = _render(*case, overlap=0)
    for n in (2, 3, 4):
        got, st = _render(*case, overlap=n)
        assert np.array_equal(got.view(np.uint64), one.view(np.uint64)), (n, np.abs(got - one).max())
        assert st["segments"] == st1["segments"] and st["samples"] == st1["samples"], n
        assert st["launches_intersect"] == n, n
