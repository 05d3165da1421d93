"""tiler_amd -- MI355X-native tile-search hot path of GliGli's TileMotion encoder (b0nefish/tiler).

FrameTiling exact NN (ANN.dll drop-in, libANN.so), Smooth and GlobalTiling K-Modes as hand-written
gfx950 HIP kernels behind a C-ABI (include/tiler_ann.h).  Python here is host plumbing only.
"""
from ._lib import LIB_PATH, TilerError, header_symbols, last_error, load  # noqa: F401
from .ann import KDTree  # noqa: F401
from .psyv import psyv_batch, psyv_batch_dev  # noqa: F401

__all__ = ["LIB_PATH", "TilerError", "header_symbols", "last_error", "load", "KDTree", "psyv_batch",
           "psyv_batch_dev"]
