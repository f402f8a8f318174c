"""xynet_amd — MI355X-native WebSocket frame decode (header parse + XOR unmask).

The decode path is libxyws.so (hand-written gfx950 HIP kernels behind the C-ABI
in include/xyws.h); this package is its host-side mirror of xynet's frame
interface (``xynet_amd.websocket``) plus the in-tree build (``xynet_amd.build``).
"""
from . import _lib  # noqa: F401

__all__ = ["websocket", "build"]
