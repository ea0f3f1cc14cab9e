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
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def sample_range(spp: int, world: int, rank: int) -> Tuple[int, int]:
    """Balanced contiguous split of [0, spp) -> (begin, count) for `rank`."""
    base, extra = divmod(spp, world)
    begin = rank * base + min(rank, extra)
    return begin, base + (1 if rank < extra else 0)


def render_sharded(render_fn: Callable, nx: int, ny: int, spp: int, accum, *, mode: str = "spp",
                   group=None) -> Optional[np.ndarray]:
    """Render this rank's shard with `render_fn(spp_begin, spp_count,
    row_begin, row_step, accum)` (which ADDS its sums into `accum`, a float64
    tensor of nx*ny*3 on this rank's device), reduce to rank 0 and return the
    finalised canvas there (None on other ranks)."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    accum.zero_()
    if mode == "spp":
        b, c = sample_range(spp, world, rank)
        if c:
            render_fn(b, c, 0, 1, accum)
    elif mode == "rows":
        if rank < ny:
            render_fn(0, spp, rank, world, accum)
    else:
        raise ValueError(f"unknown sharding mode {mode!r}")
    if world > 1:
        dist.reduce(accum, dst=0, group=group)
    if rank != 0:
        return None
    from .render import finalize
    return finalize(accum.detach().cpu().numpy(), nx, ny, spp)


def gpu_render_fn(device_scene, nx: int, ny: int, spp: int, max_depth: int, seed: int = 0, **kw) -> Callable:
    """render_fn for render_sharded on a GPU: the C-ABI renderer of this rank."""

    def fn(spp_begin, spp_count, row_begin, row_step, accum):
        device_scene.render_accumulate(nx, ny, spp, max_depth, seed, spp_begin=spp_begin, spp_count=spp_count,
                                       row_begin=row_begin, row_step=row_step, accum=accum, **kw)

    return fn
