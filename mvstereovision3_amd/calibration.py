"""Calibration files and the rectification set-up of Stereosystem.

Mirror of the calibration half of ``class Stereosystem`` (inc/Stereosystem.h,
src/Stereosystem.cpp) on libmvsv:

* ``loadIntrinsic`` / ``loadExtrinisic`` / ``saveIntrinsic`` / ``saveExtrinsic``
  (src/Stereosystem.cpp:326-446): cv::FileStorage YAML matrices, byte-compatible
  with the files under the reference's parameters/ (mvsv_load_intrinsic ...);
* ``initRectification`` (:193-241): cv::stereoRectify (CALIB_ZERO_DISPARITY,
  alpha 0) + cv::initUndistortRectifyMap for both cameras, display ROI =
  intersection of the two valid ROIs, intrinsics halved while binning;
* ``getRectifiedImagepair`` (:243-277): remap both images on the GPU
  (OpenCV 3.4 fixed-point bilinear) and crop to the display ROI.

The reference's Stereosystem owns two mvIMPACT cameras; here the image size
(and binning mode) is given at construction and the raw pair is passed in.
"""
from __future__ import annotations

import ctypes
import logging

import numpy as np

from . import _lib
from ._lib import MvsvError, Rect, lib

log = logging.getLogger("mvsv.stereosystem")

MAT_MAX = 16
CALIB_ZERO_DISPARITY = 1024
_DT = {"u": np.uint8, "c": np.int8, "w": np.uint16, "s": np.int16, "i": np.int32,
       "f": np.float32, "d": np.float64}


class Mat(ctypes.Structure):
    """mvsv_mat: up to 16 elements, rows = cols = 0 for an empty matrix (dt 'u')."""
    _fields_ = [("rows", ctypes.c_int), ("cols", ctypes.c_int), ("dt", ctypes.c_char),
                ("data", ctypes.c_double * MAT_MAX)]

    @staticmethod
    def of(a, dt=None) -> "Mat":
        m = Mat()
        if a is None or np.asarray(a).size == 0:
            m.rows = m.cols = 0
            m.dt = b"u"
            return m
        arr = np.asarray(a)
        if arr.ndim == 1:
            arr = arr.reshape(-1, 1)
        if arr.ndim != 2 or arr.size > MAT_MAX:
            raise MvsvError(_lib.MVSV_E_INVALID_ARG, "matrix must be 2-D with <= 16 elements")
        if dt is None:
            dt = {np.dtype(v): k for k, v in _DT.items()}.get(arr.dtype, "d")
        m.rows, m.cols = arr.shape
        m.dt = dt.encode()
        for i, v in enumerate(arr.astype(np.float64).reshape(-1)):
            m.data[i] = float(v)
        return m

    def array(self) -> np.ndarray:
        dt = self.dt.decode() if self.dt else "u"
        n = self.rows * self.cols
        return np.array(self.data[:n], dtype=np.float64).astype(_DT.get(dt, np.float64)) \
            .reshape(self.rows, self.cols)


class Intrinsics(ctypes.Structure):
    _fields_ = [(n, Mat) for n in ("camera_matrix_left", "camera_matrix_right", "dist_coeffs_left",
                                   "dist_coeffs_right", "camera_matrix_left_new",
                                   "camera_matrix_right_new", "q_matrix")]


class Extrinsics(ctypes.Structure):
    _fields_ = [(n, Mat) for n in ("R", "T", "E", "F")]


def _declare():
    L = lib()
    if getattr(L, "_calib_declared", False):
        return L
    P, I, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    S = ctypes.c_char_p
    for name, args, res in (
            ("mvsv_read_matrix_yaml", [S, S, P], I),
            ("mvsv_write_matrices_yaml", [S, P, P, I], I),
            ("mvsv_load_intrinsic", [S, P], I),
            ("mvsv_load_extrinsic", [S, P], I),
            ("mvsv_save_intrinsic", [S, P], I),
            ("mvsv_save_extrinsic", [S, P], I),
            ("mvsv_stereo_rectify", [P, P, I, P, P, I, I, I, P, P, I, D, P, P, P, P, P, P, P], I)):
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    L._calib_declared = True
    return L


def read_matrix(path, key):
    """cv::FileStorage fs[key] >> Mat for a matrix node: (array, dt)."""
    m = Mat()
    _lib.check(_declare().mvsv_read_matrix_yaml(str(path).encode(), key.encode(), ctypes.byref(m)))
    return m.array(), (m.dt.decode() if m.dt else "u")


def write_matrices(path, items):
    """cv::FileStorage WRITE + fs << key << mat for each (key, array[, dt]) in order."""
    keys = (ctypes.c_char_p * len(items))(*[it[0].encode() for it in items])
    mats = (Mat * len(items))(*[Mat.of(it[1], it[2] if len(it) > 2 else None) for it in items])
    _lib.check(_declare().mvsv_write_matrices_yaml(str(path).encode(), keys, mats, len(items)))


def _d(a, n):
    a = np.ascontiguousarray(np.asarray(a, np.float64).reshape(-1))
    if a.size != n:
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, f"expected {n} values, got {a.size}")
    return a


def stereo_rectify(K1, D1, K2, D2, size, R, T, flags=CALIB_ZERO_DISPARITY, alpha=0.0):
    """cv::stereoRectify -> (R1, R2, P1, P2, Q, roi1, roi2), ROIs as (x0, y0, x1, y1)."""
    W, H = size
    K1, K2, R, T = _d(K1, 9), _d(K2, 9), _d(R, 9), _d(T, 3)
    D1 = np.ascontiguousarray(np.asarray(D1, np.float64).reshape(-1))
    D2 = np.ascontiguousarray(np.asarray(D2, np.float64).reshape(-1))
    R1, R2 = np.zeros(9), np.zeros(9)
    P1, P2, Q = np.zeros(12), np.zeros(12), np.zeros(16)
    r1, r2 = Rect(), Rect()
    ptr = lambda a: a.ctypes.data  # noqa: E731
    _lib.check(_declare().mvsv_stereo_rectify(
        ptr(K1), ptr(D1) if D1.size else None, D1.size, ptr(K2), ptr(D2) if D2.size else None,
        D2.size, W, H, ptr(R), ptr(T), flags, alpha, ptr(R1), ptr(R2), ptr(P1), ptr(P2), ptr(Q),
        ctypes.byref(r1), ctypes.byref(r2)))
    return (R1.reshape(3, 3), R2.reshape(3, 3), P1.reshape(3, 4), P2.reshape(3, 4),
            Q.reshape(4, 4), (r1.x0, r1.y0, r1.x1, r1.y1), (r2.x0, r2.y0, r2.x1, r2.y1))


class Stereosystem:
    """Calibration / rectification part of Stereosystem (inc/Stereosystem.h:16-86)."""

    def __init__(self, width, height, binning=False):
        self.mTag = "STEREOSYSTEM\t"
        self.width, self.height, self.binning = int(width), int(height), bool(binning)
        self.mIntrinsicLeft = self.mIntrinsicRight = None
        self.mDistCoeffsLeft = self.mDistCoeffsRight = None
        self.mR = self.mT = self.mE = self.mF = None
        self.mR0 = self.mR1 = self.mP0 = self.mP1 = self.mQ = None
        self.mMap1 = [None, None]
        self.mMap2 = [None, None]
        self.mValidROI = [None, None]
        self.mDisplayROI = None
        self.mIsInit = False

    # --- load / save (src/Stereosystem.cpp:326-446) ---------------------------
    def loadIntrinsic(self, file) -> bool:
        v = Intrinsics()
        rc = _declare().mvsv_load_intrinsic(str(file).encode(), ctypes.byref(v))
        if rc == _lib.MVSV_E_PARSE:
            log.error("%sNode in %s is empty.", self.mTag, file)
            return False
        if rc < 0:
            log.error("%sUnable to open intrinsic file: %s", self.mTag, file)
            return False
        self.mIntrinsicLeft = v.camera_matrix_left.array()
        self.mIntrinsicRight = v.camera_matrix_right.array()
        self.mDistCoeffsLeft = v.dist_coeffs_left.array()
        self.mDistCoeffsRight = v.dist_coeffs_right.array()
        log.info("%sSuccessfully loaded Intrinsics.", self.mTag)
        return True

    def loadExtrinisic(self, file) -> bool:  # sic: the reference's spelling
        v = Extrinsics()
        rc = _declare().mvsv_load_extrinsic(str(file).encode(), ctypes.byref(v))
        if rc == _lib.MVSV_E_PARSE:
            log.error("%sNode in %sis empty.", self.mTag, file)
            return False
        if rc < 0:
            log.error("%sUnable to open extrinsic file: %s", self.mTag, file)
            return False
        self.mR, self.mT, self.mE, self.mF = v.R.array(), v.T.array(), v.E.array(), v.F.array()
        log.info("%sSuccessfully loaded Extrinsics.", self.mTag)
        return True

    def saveIntrinsic(self, file) -> bool:
        v = Intrinsics(Mat.of(self.mIntrinsicLeft), Mat.of(self.mIntrinsicRight),
                       Mat.of(self.mDistCoeffsLeft), Mat.of(self.mDistCoeffsRight),
                       Mat.of(self.mP0), Mat.of(self.mP1), Mat.of(self.mQ))
        if _declare().mvsv_save_intrinsic(str(file).encode(), ctypes.byref(v)) < 0:
            log.error("%sUnable to open %s for saving.", self.mTag, file)
            return False
        return True

    def saveExtrinsic(self, file) -> bool:
        v = Extrinsics(Mat.of(self.mR), Mat.of(self.mT), Mat.of(self.mE), Mat.of(self.mF))
        if _declare().mvsv_save_extrinsic(str(file).encode(), ctypes.byref(v)) < 0:
            log.error("%sUnable to open %s for saving.", self.mTag, file)
            return False
        return True

    # --- getters (src/Stereosystem.cpp:40-80) ---------------------------------
    def getFundamentalMatrix(self):
        return self.mF

    def getTranslationMatrix(self):
        return self.mT

    def getBaseline(self) -> float:
        t = np.asarray(self.mT, np.float64).reshape(-1)
        return float(np.sqrt(t[0] ** 2 + t[1] ** 2 + t[2] ** 2))

    def getRotationMatrix(self):
        return self.mR

    def getQMatrix(self):
        return self.mQ

    def getNewKMats(self):
        return [self.mP0, self.mP1]

    # --- rectification (src/Stereosystem.cpp:193-277) --------------------------
    def initRectification(self) -> bool:
        from .rectify import init_undistort_rectify_map
        if self.mIntrinsicLeft is None or self.mR is None:
            log.error("%sUnable to init rectification", self.mTag)
            return False
        KL = np.asarray(self.mIntrinsicLeft, np.float64)
        KR = np.asarray(self.mIntrinsicRight, np.float64)
        if self.binning:
            KL, KR = KL / 2, KR / 2
        size = (self.width, self.height)
        R0, R1, P0, P1, Q, roi0, roi1 = stereo_rectify(
            KL, self.mDistCoeffsLeft, KR, self.mDistCoeffsRight, size, self.mR, self.mT,
            CALIB_ZERO_DISPARITY, 0.0)
        self.mR0, self.mR1, self.mP0, self.mP1, self.mQ = R0, R1, P0, P1, Q
        self.mValidROI = [roi0, roi1]
        dl = np.asarray(self.mDistCoeffsLeft, np.float64).reshape(-1)
        dr = np.asarray(self.mDistCoeffsRight, np.float64).reshape(-1)
        self.mMap1[0], self.mMap2[0] = init_undistort_rectify_map(KL, dl, R0, P0[:, :3], size)
        self.mMap1[1], self.mMap2[1] = init_undistort_rectify_map(KR, dr, R1, P1[:, :3], size)
        self.mDisplayROI = (max(roi0[0], roi1[0]), max(roi0[1], roi1[1]),
                            min(roi0[2], roi1[2]), min(roi0[3], roi1[3]))
        log.info("%sRectification successfully initialized! %s", self.mTag, self.mDisplayROI)
        self.mIsInit = True
        return True

    def resetRectification(self):
        self.mIsInit = False

    def getRectifiedImagepair(self, sip, factor=None) -> bool:
        """Remap sip.mLeft / sip.mRight (the raw pair) on the GPU and crop to the
        display ROI; with ``factor`` (the (Stereopair&, float) overload,
        src/Stereosystem.cpp:279-315) the cropped pair is then cv::resize'd by
        it -- only when the rectification was already initialised: the
        reference's first call (which initialises) returns the unresized crop."""
        from .rectify import rectify_pair, resize
        was_init = self.mIsInit
        if not self.mIsInit and not self.initRectification():
            return False
        maps = (self.mMap1[0], self.mMap2[0], self.mMap1[1], self.mMap2[1])
        sip.mLeft, sip.mRight = rectify_pair(sip.mLeft, sip.mRight, maps, self.mDisplayROI)
        if factor is not None and was_init:
            f = float(np.float32(factor))  # the reference's float parameter
            sip.mLeft, sip.mRight = resize(sip.mLeft, f, f), resize(sip.mRight, f, f)
        return True
