"""mvstereovision3_amd — MI355X-native stereo disparity engine.

Drop-in for the disparity hot path of hG3n/mvStereoVision3
(Disparity::sgbm / Disparity::bm / Disparity::loadSGBMParameters,
src/disparity.cpp:6-108).  Compute lives in hand-written HIP kernels for
gfx950 behind the C ABI of libmvsv.so (include/mvsv.h); this package is the
host-side mirror of the reference interface.
"""
from ._lib import (MODE_HH, MODE_SGBM, MVSV_E_TIMEOUT, OPT_BITSLICE, OPT_BM_TILE_ROWS, OPT_PATH_SCHEDULE,
                   OPT_STRIP_SPIN_LIMIT, OPT_STRIP_WAVES,
                   PREFILTER_NORMALIZED_RESPONSE, PREFILTER_XSOBEL, VARIANT_FIRSTCOL_FIX,
                   VARIANT_WTA_MIN_D, MvsvError, set_option, synchronize)
from .disparity import (Disparity, StereoBM, StereoSGBM, Stereopair, mean_disparity_grid,
                        sgbmParameters, synth_pair)
from .detection import DisparityStream, MeanDisparityDetection, Subimage, create_dmap_rois
from .calibration import Stereosystem, read_matrix, stereo_rectify, write_matrices
from .rectify import init_undistort_rectify_map, rectify_pair, remap
from .utility import Utility, dMapValues, ply, reproject

__all__ = [
    "Disparity", "StereoBM", "StereoSGBM", "Stereopair", "sgbmParameters", "MvsvError",
    "synth_pair", "mean_disparity_grid", "MODE_SGBM", "MODE_HH", "PREFILTER_XSOBEL",
    "PREFILTER_NORMALIZED_RESPONSE", "VARIANT_FIRSTCOL_FIX", "VARIANT_WTA_MIN_D",
    "DisparityStream", "MeanDisparityDetection", "Subimage", "create_dmap_rois", "Utility",
    "dMapValues", "ply", "reproject", "init_undistort_rectify_map", "rectify_pair", "remap",
    "synchronize", "set_option", "Stereosystem", "read_matrix", "write_matrices",
    "stereo_rectify", "MVSV_E_TIMEOUT", "OPT_STRIP_SPIN_LIMIT", "OPT_STRIP_WAVES", "OPT_BM_TILE_ROWS",
    "OPT_PATH_SCHEDULE", "OPT_BITSLICE",
]
__version__ = "1.0.0"
