"""MI355X-native engine for the Roaring bitmap set-algebra hot path.

Drop-in for luvk1412/RoaringBitmap's pairwise static ops and FastAggregation's
wide or/and/xor.  Bitmaps travel in the portable serialized
format; every op runs in hand-written gfx950 HIP kernels behind the C ABI of
include/roaring_mi355x.h.
"""
from ._lib import (DeviceError, IllegalArgumentException, InvalidRoaringFormat, RoaringError,  # noqa: F401
                   TruncatedInput)
from .engine import Engine  # noqa: F401
from .roaring import (BufferFastAggregation, FastAggregation, ImmutableRoaringBitmap, MutableRoaringBitmap,  # noqa: F401
                      ParallelAggregation, RoaringBitmap, batch_and_cardinality, run_optimize_many)
from .bsi import BitSliceIndexBase, ImmutableBitSliceIndex, MutableBitSliceIndex, RoaringBitmapSliceIndex  # noqa: F401

__all__ = ["RoaringBitmap", "ImmutableRoaringBitmap", "MutableRoaringBitmap", "FastAggregation", "BufferFastAggregation", "ParallelAggregation", "RoaringBitmapSliceIndex", "ImmutableBitSliceIndex",
           "MutableBitSliceIndex", "BitSliceIndexBase", "Engine", "batch_and_cardinality", "run_optimize_many",
           "InvalidRoaringFormat",
           "TruncatedInput", "IllegalArgumentException", "DeviceError", "RoaringError"]
