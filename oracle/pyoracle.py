"""ctypes binding of the C oracle (oracle/build/libmvsv_oracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker / CPU baseline.  Never imported by
the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libmvsv_oracle.so")
_lib = None

SGBM_FIELDS = ("min_disparity", "num_disparities", "block_size", "p1", "p2",
               "disp12_max_diff", "pre_filter_cap", "uniqueness_ratio",
               "speckle_window_size", "speckle_range", "mode")
BM_FIELDS = ("pre_filter_type", "pre_filter_size", "pre_filter_cap", "block_size",
             "min_disparity", "num_disparities", "texture_threshold",
             "uniqueness_ratio", "speckle_window_size", "speckle_range",
             "disp12_max_diff")


class SgbmParams(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int) for f in SGBM_FIELDS]


class BmParams(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int) for f in BM_FIELDS]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "mvsv_oracle.c")
        if (not os.path.exists(_LIB_PATH)
                or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        I = ctypes.c_int
        S = ctypes.c_ssize_t
        for name in ("orc_sgbm_compute", "orc_sgbm_core"):
            f = getattr(_lib, name)
            f.argtypes = [P, S, P, S, I, I, P, ctypes.c_uint, P, S]
            f.restype = I
        _lib.orc_sgbm_cost_volume.argtypes = [P, S, P, S, I, I, P, ctypes.c_uint, P]
        _lib.orc_sgbm_cost_volume.restype = I
        _lib.orc_bm_compute.argtypes = [P, S, P, S, I, I, P, P, S]
        _lib.orc_bm_compute.restype = I
        _lib.orc_prefilter_xsobel.argtypes = [P, S, I, I, I, P]
        _lib.orc_median3x3_s16.argtypes = [P, S, I, I, P, S]
        _lib.orc_filter_speckles_s16.argtypes = [P, S, I, I, I, I, I]
        _lib.orc_filter_speckles_s16.restype = I
        _lib.orc_mean_disparity_grid.argtypes = [P, S, I, I, P]
        _lib.orc_reproject.argtypes = [P, S, I, I, P, P]
        _lib.orc_remap_linear.argtypes = [P, S, I, I, P, P, P, I, I]
        _lib.orc_resize_linear.argtypes = [P, S, I, I, ctypes.c_double, ctypes.c_double, P, S,
                                           ctypes.POINTER(I), ctypes.POINTER(I)]
    return _lib


def _u8(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def sgbm_params(p: dict) -> SgbmParams:
    return SgbmParams(*[int(p[f]) for f in SGBM_FIELDS])


def bm_params(p: dict) -> BmParams:
    return BmParams(*[int(p[f]) for f in BM_FIELDS])


def sgbm(L, R, p: dict, flags: int = 0, core_only: bool = False) -> np.ndarray:
    L, R = _u8(L), _u8(R)
    H, W = L.shape
    out = np.zeros((H, W), np.int16)
    prm = sgbm_params(p)
    fn = lib().orc_sgbm_core if core_only else lib().orc_sgbm_compute
    rc = fn(_ptr(L), W, _ptr(R), W, W, H, ctypes.byref(prm), flags, _ptr(out), W)
    if rc < 0:
        raise ValueError(f"oracle sgbm rc={rc}")
    return out


def sgbm_cost_volume(L, R, p: dict, flags: int = 0) -> np.ndarray:
    L, R = _u8(L), _u8(R)
    H, W = L.shape
    maxD = p["min_disparity"] + p["num_disparities"]
    W1 = (W + min(p["min_disparity"], 0)) - max(maxD, 0)
    C = np.zeros((H, max(W1, 0), p["num_disparities"]), np.int16)
    prm = sgbm_params(p)
    rc = lib().orc_sgbm_cost_volume(_ptr(L), W, _ptr(R), W, W, H, ctypes.byref(prm), flags,
                                    _ptr(C))
    if rc < 0:
        raise ValueError(f"oracle cost volume rc={rc}")
    return C


def bm(L, R, p: dict) -> np.ndarray:
    L, R = _u8(L), _u8(R)
    H, W = L.shape
    out = np.zeros((H, W), np.int16)
    prm = bm_params(p)
    rc = lib().orc_bm_compute(_ptr(L), W, _ptr(R), W, W, H, ctypes.byref(prm), _ptr(out), W)
    if rc < 0:
        raise ValueError(f"oracle bm rc={rc}")
    return out


def xsobel(img, cap: int) -> np.ndarray:
    img = _u8(img)
    H, W = img.shape
    out = np.zeros((H, W), np.uint8)
    lib().orc_prefilter_xsobel(_ptr(img), W, W, H, cap, _ptr(out))
    return out


def median3x3(d) -> np.ndarray:
    d = np.ascontiguousarray(d, dtype=np.int16)
    H, W = d.shape
    out = np.zeros_like(d)
    lib().orc_median3x3_s16(_ptr(d), W, W, H, _ptr(out), W)
    return out


def filter_speckles(d, new_val: int, max_size: int, max_diff: int) -> np.ndarray:
    d = np.ascontiguousarray(d, dtype=np.int16).copy()
    H, W = d.shape
    rc = lib().orc_filter_speckles_s16(_ptr(d), W, W, H, new_val, max_size, max_diff)
    if rc < 0:
        raise ValueError("oracle speckle failure")
    return d


def mean_disparity_grid(d) -> np.ndarray:
    d = np.ascontiguousarray(d, dtype=np.int16)
    H, W = d.shape
    out = np.zeros(81, np.float32)
    lib().orc_mean_disparity_grid(_ptr(d), W, W, H, _ptr(out))
    return out


def reproject(dmap: np.ndarray, Q) -> np.ndarray:
    """Utility::calcCoordinate per pixel -> (H, W, 4) float32 (X, Y, Z, valid)."""
    d = np.ascontiguousarray(dmap, np.int16)
    H, W = d.shape
    q = np.ascontiguousarray(np.asarray(Q, np.float32).reshape(16))
    out = np.empty((H, W, 4), np.float32)
    lib().orc_reproject(_ptr(d), W, W, H, _ptr(q), _ptr(out))
    return out


def remap_linear(src: np.ndarray, mapx: np.ndarray, mapy: np.ndarray) -> np.ndarray:
    """cv::remap(INTER_LINEAR, BORDER_CONSTANT 0) of a uint8 image with float32 maps."""
    s = np.ascontiguousarray(src, np.uint8)
    mx = np.ascontiguousarray(mapx, np.float32)
    my = np.ascontiguousarray(mapy, np.float32)
    dh, dw = mx.shape
    out = np.empty((dh, dw), np.uint8)
    lib().orc_remap_linear(_ptr(s), s.shape[1], s.shape[1], s.shape[0], _ptr(mx), _ptr(my),
                           _ptr(out), dw, dh)
    return out


def resize_linear(src: np.ndarray, fx: float, fy: float) -> np.ndarray:
    """cv::resize(src, dst, Size(0, 0), fx, fy, INTER_LINEAR) of a uint8 image."""
    s = np.ascontiguousarray(src, np.uint8)
    w, h = ctypes.c_int(), ctypes.c_int()
    lib().orc_resize_linear(_ptr(s), s.shape[1], s.shape[1], s.shape[0], fx, fy, None, 0,
                            ctypes.byref(w), ctypes.byref(h))
    out = np.empty((h.value, w.value), np.uint8)
    lib().orc_resize_linear(_ptr(s), s.shape[1], s.shape[1], s.shape[0], fx, fy, _ptr(out),
                            w.value, ctypes.byref(w), ctypes.byref(h))
    return out
