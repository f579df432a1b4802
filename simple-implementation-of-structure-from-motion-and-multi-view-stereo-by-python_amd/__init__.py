"""MI355X-native drop-in for the MVS patch-expansion stage of
MarvinChung/simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python.

Import with importlib (the directory name is not an identifier):
    mvs = importlib.import_module(
        "simple-implementation-of-structure-from-motion-and-multi-view-stereo-by-python_amd")
"""
from . import _lib, sfm, synthetic, utils  # noqa: F401
from ._lib import MvsContext, ncc_windows, rodrigues_roundtrip, triangulate  # noqa: F401
from .MVS2 import DensePointsWithMVS2, MyPatch, photo_consistency_batch  # noqa: F401
from .utils import SeedSet, export2ply, read_imgs, read_pars, read_ply  # noqa: F401

PACKAGE = __name__
