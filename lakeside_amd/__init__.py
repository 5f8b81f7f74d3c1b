"""lakeside_amd: MI355X-native sealed-segment DataExpr evaluator (drop-in for lakeside's worker evaluator).

The compute path is liblakeside_gpu.so (hand-written HIP kernels for gfx950 behind the C ABI in
include/lakeside_gpu.h).  Python here is the host-side mirror used by tests and the bench.
"""
from ._lib import LK_MERGED, LK_PER_GLOB_ROWS, LK_PLAN_BYTES, LakesideError  # noqa: F401

__all__ = ["LK_MERGED", "LK_PER_GLOB_ROWS", "LK_PLAN_BYTES", "LakesideError", "Engine", "evaluate_push_down_request"]


def __getattr__(name):
    if name in ("Engine", "Result", "evaluate_push_down_request"):
        from . import evaluator
        return getattr(evaluator, name)
    raise AttributeError(name)
