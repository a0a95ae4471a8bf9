"""haag_vq — MI355X-native (gfx950) build of the vector-quantization hot path.

Module paths mirror the reference package (/root/reference/src/haag_vq) so it drops in behind
the same callers; the encode / decode / search work runs in libmivq.so (HIP kernels,
include/mivq.h).  Importing the package needs no GPU; compute calls do.
"""

__version__ = "0.1.0"
