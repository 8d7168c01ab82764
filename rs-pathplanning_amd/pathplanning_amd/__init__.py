"""pathplanning_amd — MI355X-native drop-in for tsturzl/rs-pathplanning's RRT extend hot path.

``dubins`` and ``rrt`` mirror the crate's two public modules (src/lib.rs:5-6); the compute runs in
hand-written HIP kernels for gfx950 behind the C ABI in include/pathplanning_amd.h.
"""
from . import _ffi, dubins, rrt, scenes  # noqa: F401
from ._ffi import Context, PPError, device_count  # noqa: F401

__all__ = ["dubins", "rrt", "scenes", "Context", "PPError", "device_count"]
