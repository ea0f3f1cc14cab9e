"""Multi-GPU rendering: one process per GPU, torch.distributed over RCCL.

Samples are independent (the RNG is keyed by (seed, pixel, sample)), so a
render shards with no exchange during the trace; the only collective is one
reduce of the per-pixel fp64 radiance sums to rank 0 at the end
(RayTracingWeekend.cpp:235-239 is a per-pixel sum).

Two shardings:
  "spp"   rank r renders the contiguous sample range r of every pixel (every
          GPU sees the same pixel-cost mix, so the load is balanced); the
          reduce sums partial sums, which reorders the fp64 additions
          (~1e-16 relative).
  "rows"  rank r renders every pixel row j = r (mod world) with all samples;
          the reduce only assembles disjoint rows, so the result is
          bit-identical to a single-GPU render.

`render_step` is the one step both bench.py (GPU ranks over RCCL) and
tests/test_distributed.py (gloo ranks on the CPU, the oracle standing in for
each rank's renderer) run.  A C/C++ host without torch uses rtw_render_multi
(include/rtw_gpu.h) instead: one process, one thread per GPU, RCCL inside.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def sample_range(spp: int, world: int, rank: int) -> Tuple[int, int]:
    """Balanced contiguous split of [0, spp) -> (begin, count) for `rank`
    (the split rtw_render_multi uses too)."""
    base, extra = divmod(spp, world)
    begin = rank * base + min(rank, extra)
    return begin, base + (1 if rank < extra else 0)


def _world(group):
    import torch.distributed as dist
    if not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


PHASES = ("render", "reduce", "finalize")


def render_step(render_fn: Callable, finalize_fn: Optional[Callable], accum, canvas, nx: int, ny: int, spp: int, *,
                mode: str = "spp", group=None, timings: Optional[dict] = None, sync: Optional[Callable] = None):
    """One render of the whole image by every rank of `group`:

      accum <- 0; render_fn(spp_begin, spp_count, row_begin, row_step, accum)
      ADDS this rank's shard of the per-pixel sums; dist.reduce(SUM) to rank 0;
      on rank 0 finalize_fn(accum, canvas) writes min(sqrt(accum / spp), 1)
      (RayTracingWeekend.cpp:241-244).

    timings: when given, the wall milliseconds of this rank's phases are
    ADDED into it under PHASES ("render": zero + render, "reduce": the
    collective, "finalize"), each closed by `sync()` (torch.cuda.synchronize
    on a GPU) so that queued device work is counted in its own phase.

    Returns render_fn's result on this rank (its stats), or None when the
    rank had no shard."""
    import time

    import torch.distributed as dist

    world, rank = _world(group)
    t = [time.perf_counter()]

    def mark():
        if timings is not None:
            if sync is not None:
                sync()
            t.append(time.perf_counter())

    accum.zero_()
    out = None
    if mode == "spp":
        b, c = sample_range(spp, world, rank)
        if c:
            out = render_fn(b, c, 0, 1, accum)
    elif mode == "rows":
        if rank < ny:
            out = render_fn(0, spp, rank, world, accum)
    else:
        raise ValueError(f"unknown sharding mode {mode!r}")
    mark()
    if world > 1:
        dist.reduce(accum, dst=0, group=group)
    mark()
    if rank == 0 and finalize_fn is not None:
        finalize_fn(accum, canvas)
    mark()
    if timings is not None:
        for k, name in enumerate(PHASES):
            timings[name] = timings.get(name, 0.0) + (t[k + 1] - t[k]) * 1e3
    return out


def render_sharded(render_fn: Callable, nx: int, ny: int, spp: int, accum, *, mode: str = "spp",
                   group=None) -> Optional[np.ndarray]:
    """render_step with the host finalize (rtw_finalize_canvas); returns the
    canvas as a numpy array on rank 0 (None on other ranks)."""
    from .render import finalize

    box = {}

    def fin(acc, _canvas):
        box["canvas"] = finalize(acc.detach().cpu().numpy(), nx, ny, spp)

    render_step(render_fn, fin, accum, None, nx, ny, spp, mode=mode, group=group)
    return box.get("canvas")


def gpu_render_fn(device_scene, nx: int, ny: int, spp: int, max_depth: int, seed: int = 0, **kw) -> Callable:
    """render_fn for render_step on a GPU: the C-ABI renderer of this rank
    (returns its rtw_stats as a dict)."""

    def fn(spp_begin, spp_count, row_begin, row_step, accum):
        _, st = device_scene.render_accumulate(nx, ny, spp, max_depth, seed, spp_begin=spp_begin,
                                               spp_count=spp_count, row_begin=row_begin, row_step=row_step,
                                               accum=accum, **kw)
        return st

    return fn


def gpu_finalize_fn(device_scene, nx: int, ny: int, spp: int) -> Callable:
    """finalize_fn for render_step on a GPU: rtw_finalize_canvas_device."""

    def fn(accum, canvas):
        device_scene.finalize_device(accum, nx, ny, spp, canvas)

    return fn
