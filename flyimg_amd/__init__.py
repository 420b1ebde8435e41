"""flyimg_amd -- MI355X (gfx950) image hot path of flyimg behind its own
processor / smartcrop interfaces.

The product is the C-ABI library ``libflyimg_hip.so`` (include/flyimg_hip.h,
hand-written HIP kernels in csrc/).  This package holds its ctypes binding
(_lib, runtime), the host-side mirror of the reference's option model and
ImageProcessor (processor), the drop-in smartcrop module (smartcrop), the
seeded synthetic image generator (synth) and the multi-rank plumbing
(parallel).  Nothing here falls back to CPU pixel code.
"""
from . import _lib  # noqa: F401

__all__ = ["_lib", "runtime", "processor", "smartcrop", "synth", "parallel"]
