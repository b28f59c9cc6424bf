"""Host-side mirror of the reference's disparity interface, on libmvsv.

Reference surface (hG3n/mvStereoVision3):

* ``struct Stereopair``                inc/utility.h:31-41
* ``Disparity::sgbmParameters``        inc/disparity.h:17-27
* ``Disparity::sgbm(Stereopair const&, cv::Mat&, cv::Ptr<cv::StereoSGBM>)``
                                       src/disparity.cpp:6-10
* ``Disparity::bm(Stereopair const&, cv::Mat&, cv::Ptr<cv::StereoBM>)``
                                       src/disparity.cpp:18-22
* ``Disparity::loadSGBMParameters(std::string, cv::Ptr<cv::StereoSGBM>&,
  sgbmParameters&) -> bool``           src/disparity.cpp:60-108
* the matcher objects themselves: ``cv::StereoSGBM::create(...)`` /
  ``cv::StereoBM::create(...)`` plus their setters (src/disparity.cpp:83-95,
  trgt/liveDisparity.cpp:61, trgt/captureDisparity.cpp:196).

Same names, same argument meaning, same error behaviour: invalid matcher state
raises (OpenCV raises ``cv::Exception``; here :class:`MvsvError`), the loader
returns ``False``.  Images are host ``numpy`` uint8 arrays (ROI views with
stride > width are accepted, like the cropped ``cv::Mat`` of
src/Stereosystem.cpp:255-256) or HBM-resident ``torch`` uint8 tensors; the
result is int16 disparity x 16 (CV_16S).  All compute runs in the HIP kernels
of libmvsv.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import logging
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import (MODE_HH, MODE_SGBM, PREFILTER_NORMALIZED_RESPONSE, PREFILTER_XSOBEL,
                   BmParams, MvsvError, SgbmParams, SgbmYamlValues, check, context, lib)

log = logging.getLogger("mvsv.disparity")

DISP_SHIFT = 4
DISP_SCALE = 1 << DISP_SHIFT


@dataclass
class Stereopair:
    """inc/utility.h:31-41 — a rectified left/right pair plus a log tag."""
    mLeft: object = None
    mRight: object = None
    mTag: str = field(default="STEREOPAIR\t")


@dataclass
class sgbmParameters:  # noqa: N801 - reference name
    """Disparity::sgbmParameters, inc/disparity.h:17-27."""
    minDisp: int = 0
    numDisp: int = 0
    blockSize: int = 0
    disp12MaxDiff: int = 0
    preFilterCap: int = 0
    uniquenessRatio: int = 0
    speckleWindowSize: int = 0
    speckleRange: int = 0
    disparityMode: int = 0


def _is_torch(a) -> bool:
    return type(a).__module__.startswith("torch")


def _run_host(fn, params, left, right, out, what):
    L = np.asarray(left)
    R = np.asarray(right)
    if L.ndim != 2 or R.ndim != 2 or L.dtype != np.uint8 or R.dtype != np.uint8:
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, f"{what}: inputs must be 2-D CV_8UC1 (uint8)")
    if L.shape != R.shape:
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, f"{what}: left and right sizes differ")
    if L.strides[1] != 1:
        L = np.ascontiguousarray(L)
    if R.strides[1] != 1:
        R = np.ascontiguousarray(R)
    H, W = L.shape
    if out is None or not isinstance(out, np.ndarray) or out.shape != (H, W) \
            or out.dtype != np.int16 or out.strides[1] != 2:
        out = np.empty((H, W), np.int16)  # cv::Mat::create semantics: reallocate
    ctx = context(0)
    check(lib().mvsv_use_own_stream(ctx.handle), ctx.handle)
    rc = fn(ctx.handle, L.ctypes.data, L.strides[0], R.ctypes.data, R.strides[0], W, H,
            ctypes.byref(params), out.ctypes.data, out.strides[0] // 2)
    check(rc, ctx.handle)
    return out


def _run_device(fn, params, left, right, out, what):
    import torch
    if left.dtype != torch.uint8 or right.dtype != torch.uint8:
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, f"{what}: inputs must be uint8")
    if left.shape != right.shape or left.dim() not in (2, 3):
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, f"{what}: inputs must be (H,W) or (N,H,W), equal")
    if not left.is_cuda or not right.is_cuda or left.device != right.device:
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, f"{what}: device tensors on one GPU expected")
    batched = left.dim() == 3
    Lt = left if batched else left.unsqueeze(0)
    Rt = right if batched else right.unsqueeze(0)
    if Lt.stride(2) != 1:
        Lt = Lt.contiguous()
    if Rt.stride(2) != 1:
        Rt = Rt.contiguous()
    n, H, W = Lt.shape
    if out is None or tuple(out.shape) != tuple(left.shape) or out.dtype != torch.int16 \
            or out.device != left.device or out.stride(-1) != 1:
        out = torch.empty(left.shape, dtype=torch.int16, device=left.device)
    Ot = out if batched else out.unsqueeze(0)
    dev = left.device.index or 0
    ctx = context(dev)
    stream = torch.cuda.current_stream(left.device).cuda_stream
    check(lib().mvsv_set_stream(ctx.handle, ctypes.c_void_p(stream)), ctx.handle)
    rc = fn(ctx.handle, n, Lt.data_ptr(), Lt.stride(1), Lt.stride(0), Rt.data_ptr(), Rt.stride(1),
            Rt.stride(0), W, H, ctypes.byref(params), Ot.data_ptr(), Ot.stride(1), Ot.stride(0))
    check(rc, ctx.handle)
    return out


class StereoMatcher:
    DISP_SHIFT = DISP_SHIFT
    DISP_SCALE = DISP_SCALE

    def compute(self, left, right, disparity=None):
        """cv::StereoMatcher::compute: returns the CV_16S disparity map."""
        if _is_torch(left):
            return _run_device(self._dev_fn(), self._params, left, right, disparity,
                               type(self).__name__)
        return _run_host(self._host_fn(), self._params, left, right, disparity,
                         type(self).__name__)

    # common setters / getters of cv::StereoMatcher
    def setMinDisparity(self, v): self._params.min_disparity = int(v)      # noqa: E704
    def getMinDisparity(self): return self._params.min_disparity            # noqa: E704
    def setNumDisparities(self, v): self._params.num_disparities = int(v)  # noqa: E704
    def getNumDisparities(self): return self._params.num_disparities        # noqa: E704
    def setBlockSize(self, v): self._params.block_size = int(v)            # noqa: E704
    def getBlockSize(self): return self._params.block_size                  # noqa: E704
    def setSpeckleWindowSize(self, v): self._params.speckle_window_size = int(v)  # noqa: E704
    def getSpeckleWindowSize(self): return self._params.speckle_window_size       # noqa: E704
    def setSpeckleRange(self, v): self._params.speckle_range = int(v)       # noqa: E704
    def getSpeckleRange(self): return self._params.speckle_range            # noqa: E704
    def setDisp12MaxDiff(self, v): self._params.disp12_max_diff = int(v)   # noqa: E704
    def getDisp12MaxDiff(self): return self._params.disp12_max_diff         # noqa: E704

    def params(self) -> dict:
        return self._params.as_dict()


class StereoSGBM(StereoMatcher):
    """cv::StereoSGBM (OpenCV 3.4 semantics) backed by the MI355X kernels."""
    MODE_SGBM = MODE_SGBM
    MODE_HH = MODE_HH

    def __init__(self, params: SgbmParams):
        self._params = params

    @staticmethod
    def create(minDisparity=0, numDisparities=16, blockSize=3, P1=0, P2=0, disp12MaxDiff=0,
               preFilterCap=0, uniquenessRatio=0, speckleWindowSize=0, speckleRange=0,
               mode=MODE_SGBM):
        p = SgbmParams()
        lib().mvsv_sgbm_params_create(ctypes.byref(p), int(minDisparity), int(numDisparities),
                                      int(blockSize), int(P1), int(P2), int(disp12MaxDiff),
                                      int(preFilterCap), int(uniquenessRatio),
                                      int(speckleWindowSize), int(speckleRange), int(mode))
        return StereoSGBM(p)

    def _host_fn(self): return lib().mvsv_sgbm         # noqa: E704
    def _dev_fn(self): return lib().mvsv_sgbm_device   # noqa: E704

    def setPreFilterCap(self, v): self._params.pre_filter_cap = int(v)      # noqa: E704
    def getPreFilterCap(self): return self._params.pre_filter_cap            # noqa: E704
    def setUniquenessRatio(self, v): self._params.uniqueness_ratio = int(v)  # noqa: E704
    def getUniquenessRatio(self): return self._params.uniqueness_ratio       # noqa: E704
    def setP1(self, v): self._params.p1 = int(v)                             # noqa: E704
    def getP1(self): return self._params.p1                                  # noqa: E704
    def setP2(self, v): self._params.p2 = int(v)                             # noqa: E704
    def getP2(self): return self._params.p2                                  # noqa: E704
    def setMode(self, v): self._params.mode = int(v)                         # noqa: E704
    def getMode(self): return self._params.mode                              # noqa: E704
    def setVariant(self, v): self._params.variant = int(v)                   # noqa: E704


class StereoBM(StereoMatcher):
    """cv::StereoBM (OpenCV 3.4 semantics, CV_16S output) on the MI355X kernels."""
    PREFILTER_NORMALIZED_RESPONSE = PREFILTER_NORMALIZED_RESPONSE
    PREFILTER_XSOBEL = PREFILTER_XSOBEL

    def __init__(self, params: BmParams):
        self._params = params

    @staticmethod
    def create(numDisparities=0, blockSize=21):
        p = BmParams()
        lib().mvsv_bm_params_default(ctypes.byref(p), int(numDisparities), int(blockSize))
        return StereoBM(p)

    def _host_fn(self): return lib().mvsv_bm           # noqa: E704
    def _dev_fn(self): return lib().mvsv_bm_device     # noqa: E704

    def setPreFilterType(self, v): self._params.pre_filter_type = int(v)     # noqa: E704
    def getPreFilterType(self): return self._params.pre_filter_type          # noqa: E704
    def setPreFilterSize(self, v): self._params.pre_filter_size = int(v)     # noqa: E704
    def getPreFilterSize(self): return self._params.pre_filter_size          # noqa: E704
    def setPreFilterCap(self, v): self._params.pre_filter_cap = int(v)       # noqa: E704
    def getPreFilterCap(self): return self._params.pre_filter_cap            # noqa: E704
    def setTextureThreshold(self, v): self._params.texture_threshold = int(v)  # noqa: E704
    def getTextureThreshold(self): return self._params.texture_threshold       # noqa: E704
    def setUniquenessRatio(self, v): self._params.uniqueness_ratio = int(v)    # noqa: E704
    def getUniquenessRatio(self): return self._params.uniqueness_ratio         # noqa: E704


class Disparity:
    """namespace Disparity (inc/disparity.h:15-36)."""

    sgbmParameters = sgbmParameters

    @staticmethod
    def sgbm(inputImages: Stereopair, output, dispCompute: StereoSGBM):
        """src/disparity.cpp:6-10: forwards to compute(); returns the (re)allocated map."""
        return dispCompute.compute(inputImages.mLeft, inputImages.mRight, output)

    @staticmethod
    def bm(inputImages: Stereopair, output, dispCompute: StereoBM):
        """src/disparity.cpp:18-22."""
        return dispCompute.compute(inputImages.mLeft, inputImages.mRight, output)

    @staticmethod
    def loadSGBMParameters(filename: str, disparityObj: StereoSGBM,
                           para: sgbmParameters) -> bool:
        """src/disparity.cpp:60-108: reads configs/sgbm.yml, applies 8 setters + mode.

        P1/P2 are left untouched (programs create the matcher with P1 = P2 = 0,
        so OpenCV's effective P1 = 2, P2 = 5 apply).
        """
        vals = SgbmYamlValues()
        rc = lib().mvsv_load_sgbm_yaml(str(filename).encode(), ctypes.byref(disparityObj._params),
                                       ctypes.byref(vals))
        if rc == _lib.MVSV_E_PARSE:
            log.error("Node in %s is empty", filename)
            return False
        if rc < 0:
            log.error("Unable to open disparity parameters")
            return False
        for f in _lib.YAML_FIELDS:
            setattr(para, f, int(getattr(vals, f)))
        log.info("Successfully loaded disparity parameters")
        return True

    @staticmethod
    def loadBMParameters(filename: str, disparityObj: StereoBM) -> bool:
        """New: reads configs/bm.yml:2-7 (shipped by the reference, read by nothing)."""
        rc = lib().mvsv_load_bm_yaml(str(filename).encode(), ctypes.byref(disparityObj._params))
        if rc < 0:
            log.error("Unable to load BM parameters from %s", filename)
            return False
        return True


def synth_pair(seed: int, width: int, height: int, min_disparity: int, num_disparities: int):
    """Deterministic synthetic rectified pair; host uint8 arrays."""
    L = np.empty((height, width), np.uint8)
    R = np.empty((height, width), np.uint8)
    check(lib().mvsv_synth_pair(ctypes.c_uint32(seed & 0xFFFFFFFF), width, height,
                                min_disparity, num_disparities, L.ctypes.data, R.ctypes.data))
    return L, R


def mean_disparity_grid(dmap):
    """MeanDisparityDetection::build(MEAN_VALUE) on device: (N,81) or (81,) float32."""
    import torch
    if not _is_torch(dmap) or not dmap.is_cuda or dmap.dtype != torch.int16:
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, "mean_disparity_grid: int16 device tensor expected")
    batched = dmap.dim() == 3
    d = dmap if batched else dmap.unsqueeze(0)
    if d.stride(2) != 1:
        d = d.contiguous()
    n, H, W = d.shape
    out = torch.empty((n, 81), dtype=torch.float32, device=dmap.device)
    ctx = context(dmap.device.index or 0)
    check(lib().mvsv_set_stream(ctx.handle,
                                ctypes.c_void_p(torch.cuda.current_stream(dmap.device).cuda_stream)),
          ctx.handle)
    check(lib().mvsv_mean_disparity_grid_device(ctx.handle, n, d.data_ptr(), d.stride(1),
                                                d.stride(0), W, H, out.data_ptr()), ctx.handle)
    return out if batched else out[0]
