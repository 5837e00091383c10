"""tadpole_amd — MI355X-native engine for TADpole's per-matrix hot path.

R API mirror (reference NAMESPACE:3-8): ``TADpole``, ``load_mat``, ``diffT``,
``random_bed``.  Compute runs in ``libtadpole_hip.so`` (HIP, gfx950) through the
C ABI of ``include/tadpole_hip.h``; there is no CPU fallback.
"""
from .api import (Chclust, Mat, Tadpole, TADpole, bin_index, diffT, is_na, is_r_na, load_mat,
                  mask, random_bed, read_matrix)
from ._lib import TadpoleError

__all__ = ["TADpole", "load_mat", "diffT", "random_bed", "bin_index", "mask", "read_matrix",
           "Tadpole", "Chclust", "Mat", "TadpoleError", "is_na", "is_r_na"]
__version__ = "0.1.0"
