"""vfilter — MI355X-native backend for the per-frame filter of
kylemcdonald/distributed-video-filter (inverter.py inside worker.py, fanned out by
distributor.py).

  filters      ``bitwise_not`` (the ``cv2.bitwise_not`` drop-in, inverter.py:41) and batch forms
  _lib         ctypes binding to libvfilter_hip.so (include/vfilter.h)

The worker loop, the inverter plugin and the distributor live in ``worker``,
``inverter`` and ``distributor`` (imported on demand; they need no GPU to import).
"""
from ._lib import (ABI_VERSION, Context, VFilterError, device_count, get_context,  # noqa: F401
                   library_path, load_library)
from .filters import bitwise_not, invert, invert_batch, invert_bytes, invert_frames  # noqa: F401

__all__ = [
    "ABI_VERSION", "Context", "VFilterError", "device_count", "get_context", "library_path",
    "load_library", "bitwise_not", "invert", "invert_batch", "invert_bytes", "invert_frames",
]
