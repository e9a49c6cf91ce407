"""mahout_amd -- MI355X-native count-min-sketch ingest and sketch-cosine
similarity for Mahout Taste's CosineCM path.

The compute lives in libmahout_cms.so (hand-written gfx950 HIP kernels behind
the C ABI of include/mahout_cms.h); this package is the host-side binding and
the mirror of the reference's plugin surface (taste.CosineCM).
"""
from . import _lib  # noqa: F401
from .sketch import SketchTable, shape_from_delta_epsilon, shard_of_key, comm_unique_id  # noqa: F401

__all__ = ["SketchTable", "shape_from_delta_epsilon", "shard_of_key", "comm_unique_id"]
