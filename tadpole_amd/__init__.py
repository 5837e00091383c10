"""tadpole_amd — MI355X-native engine for TADpole's per-matrix hot path.

R API mirror (reference NAMESPACE:3-8): ``TADpole``, ``load_mat``, ``diffT``,
``random_bed``.  Compute runs in ``libtadpole_hip.so`` (HIP, gfx950) through the
C ABI of ``include/tadpole_hip.h``; there is no CPU fallback.
"""
import os as _os


def use_hw_queues(n: int = 16) -> None:
    """Opt-in: ask HIP for ``n`` hardware queues per device (GPU_MAX_HW_QUEUES).

    Concurrent pipelines (``TADpole(stream=...)``, ``run_genome``) want one
    hardware queue per stream: HIP's default is 4 and streams that share a
    queue serialise.  Importing the package changes nothing; call this (or
    export the variable) before anything initialises HIP, e.g. before
    ``import torch`` touches the GPU.  A larger value already set is kept."""
    if int(_os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < n:
        _os.environ["GPU_MAX_HW_QUEUES"] = str(int(n))


from .api import (Chclust, Mat, Tadpole, TADpole, bin_index, diffT, is_na, is_r_na, load_mat,
                  mask, random_bed, read_matrix)
from ._lib import TadpoleError, release_stream

__all__ = ["TADpole", "load_mat", "diffT", "random_bed", "bin_index", "mask", "read_matrix",
           "Tadpole", "Chclust", "Mat", "TadpoleError", "is_na", "is_r_na", "use_hw_queues",
           "release_stream"]
__version__ = "0.1.0"
