"""ecwide_amd — MI355X-native wide-stripe erasure encode / CL repair engine.

Drop-in replacement for ECWide-C's codec path (NativeCodec over ISA-L): the
product is ``libecwide.so`` (HIP kernels for gfx950 behind the C ABI in
include/ecwide.h); this package is its host-side mirror of the reference's
CodingScheme / NativeCodec interface plus the HBM stripe-slab batch API.
"""
from .codec import (BlockBatch, CodingScheme, EcwError, NativeCodec, PinnedHost, device_count,  # noqa: F401
                    get_schedule, parse_schedule, service_counters, set_schedule, xor_reduce)
from .slab import StripeSlab  # noqa: F401
from ._lib import LIB_PATH, lib  # noqa: F401

__all__ = ["CodingScheme", "NativeCodec", "EcwError", "StripeSlab", "BlockBatch", "xor_reduce", "device_count",
           "service_counters", "get_schedule", "set_schedule", "parse_schedule", "PinnedHost", "LIB_PATH"]
