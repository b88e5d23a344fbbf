"""gossip_protocol_amd -- MI355X-native gossip-membership engine.

The product is libgossip_amd.so (HIP kernels for gfx950 behind the C ABI in
include/gossip/gossip.h).  This package is the thin Python side: the ctypes binding
(_lib), the exact-mode Application mirror (exact) and the scale-mode engine (scale).
"""
from ._lib import GspError, lib  # noqa: F401

__all__ = ["GspError", "lib"]
