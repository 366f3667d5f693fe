"""goworld_amd -- MI355X-native AOI (area-of-interest) engine for GoWorld.

The one hot path accelerated here is go-aoi's XZListAOIManager as GoWorld's
engine/entity.Space drives it (Space.go:105,211,221,243,259).  The product is
the C-ABI library libgwaoi.so (include/gwaoi.h, HIP kernels for gfx950);
this package holds its ctypes binding (``_lib``), the host-side mirror of the
go-aoi interface (``aoi``), the seeded workloads (``workload``) and the
in-tree build (``build``).
"""
from ._lib import GwaoiError, Wire, World, load, pair_keys  # noqa: F401

__all__ = ["World", "Wire", "GwaoiError", "load", "pair_keys"]
