"""comet_amd — MI355X-native COMET Trajectory-Guided Temporal Modeling path.

Host code (this package) mirrors the reference comet/models operator API; every heavy op runs in
libcomet_hip.so (hand-written HIP for gfx950) through the C-ABI declared in include/comet_hip.h.
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
