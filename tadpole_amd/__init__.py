"""tadpole_amd — MI355X-native engine for TADpole's per-matrix hot path.

R API mirror (reference NAMESPACE:3-8): ``TADpole``, ``load_mat``, ``diffT``,
``random_bed``.  Compute runs in ``libtadpole_hip.so`` (HIP, gfx950) through the
C ABI of ``include/tadpole_hip.h``; there is no CPU fallback.
"""
import os as _os

# Concurrent pipelines (TADpole(stream=...), run_genome) need one hardware
# queue per stream; HIP's default is 4 and streams that share a queue
# serialise.  Raised to 16 (TADPOLE_KEEP_HW_QUEUES=1 leaves it alone); takes
# effect only if HIP has not been initialised yet.
if not _os.environ.get("TADPOLE_KEEP_HW_QUEUES") and int(_os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    _os.environ["GPU_MAX_HW_QUEUES"] = "16"

from .api import (Chclust, Mat, Tadpole, TADpole, bin_index, diffT, is_na, is_r_na, load_mat,
                  mask, random_bed, read_matrix)
from ._lib import TadpoleError

__all__ = ["TADpole", "load_mat", "diffT", "random_bed", "bin_index", "mask", "read_matrix",
           "Tadpole", "Chclust", "Mat", "TadpoleError", "is_na", "is_r_na"]
__version__ = "0.1.0"
