"""raytracingweekend_amd — an MI355X (gfx950) path tracer with the scene API of
silvesthu/RayTracingWeekend.

Native pieces (built in-tree by `python -m raytracingweekend_amd.build`):
  librtw.so     HIP wavefront kernels + the C ABI of include/rtw_gpu.h + the
                host C++ scene API (hittable / material / texture / camera /
                scene classes and the flattener)
  rtw_render    C++ host program equivalent of the reference's main()

Python: `render` (single GPU), `distributed` (one process per GPU,
torch.distributed over RCCL).
"""
from ._abi import RtwError, lib  # noqa: F401

__all__ = ["RtwError", "lib"]
