"""Rectification before the path.

Mirrors Stereosystem::initRectification (src/Stereosystem.cpp:193-237: maps from
cv::initUndistortRectifyMap, CV_32FC1) and Stereosystem::getRectifiedImagepair
(:243-262: cv::remap INTER_LINEAR on both images, then the mDisplayROI crop)
and its resizing overload (:279-315: cv::resize INTER_LINEAR by a factor).
The remap runs in a HIP kernel with OpenCV 3.4's fixed-point arithmetic
(bit-exact for given maps); the map construction is a host double-precision
restatement (OpenCV inverts P*R by SVD, so a map may differ in the last bit).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import MvsvError, Rect, check, context, lib


def init_undistort_rectify_map(K, dist, R, P, size):
    """cv::initUndistortRectifyMap(K, dist, R, P, (w, h), CV_32FC1) -> (map_x, map_y)."""
    w, h = size
    K = np.ascontiguousarray(np.asarray(K, np.float64).reshape(3, 3))
    d = np.ascontiguousarray(np.asarray(dist if dist is not None else [], np.float64).reshape(-1))
    Rm = np.ascontiguousarray(np.asarray(R if R is not None else np.eye(3), np.float64).reshape(3, 3))
    Pm = np.asarray(P, np.float64)
    Pm = np.ascontiguousarray(Pm.reshape(3, -1)[:, :3])
    mx = np.empty((h, w), np.float32)
    my = np.empty((h, w), np.float32)
    rc = lib().mvsv_init_undistort_rectify_map(K.ctypes.data, d.ctypes.data if d.size else None,
                                               int(d.size), Rm.ctypes.data, Pm.ctypes.data, w, h,
                                               mx.ctypes.data, my.ctypes.data, w)
    check(rc)
    return mx, my


def remap(src, map_x, map_y):
    """cv::remap(src, dst, map_x, map_y, INTER_LINEAR) for uint8 device tensors.

    src: (H, W) or (N, H, W) uint8 torch tensor on a HIP device; maps: float32
    device tensors of the output size.  Returns uint8 of shape (..., mh, mw).
    """
    import torch
    if not (type(src).__module__.startswith("torch") and src.is_cuda and src.dtype == torch.uint8):
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, "remap: uint8 device tensor expected")
    mx = map_x.contiguous()
    my = map_y.contiguous()
    if mx.shape != my.shape or mx.dtype != torch.float32 or mx.dim() != 2:
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, "remap: two float32 maps of one size expected")
    batched = src.dim() == 3
    s = src if batched else src.unsqueeze(0)
    if s.stride(2) != 1:
        s = s.contiguous()
    n, sh, sw = s.shape
    dh, dw = mx.shape
    out = torch.empty((n, dh, dw), dtype=torch.uint8, device=src.device)
    ctx = context(src.device.index or 0)
    check(lib().mvsv_set_stream(ctx.handle,
                                ctypes.c_void_p(torch.cuda.current_stream(src.device).cuda_stream)),
          ctx.handle)
    check(lib().mvsv_remap_device(ctx.handle, n, s.data_ptr(), s.stride(1), s.stride(0), sw, sh,
                                  mx.data_ptr(), my.data_ptr(), dw, out.data_ptr(), dw, dh * dw,
                                  dw, dh), ctx.handle)
    return out if batched else out[0]


def rectify_pair(left, right, maps, roi):
    """Stereosystem::getRectifiedImagepair on host images.

    maps = (left_x, left_y, right_x, right_y) float32 arrays of the image size;
    roi = (x0, y0, x1, y1) display ROI.  Returns the cropped rectified pair.
    """
    L = np.ascontiguousarray(left, np.uint8)
    R = np.ascontiguousarray(right, np.uint8)
    if L.shape != R.shape or L.ndim != 2:
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, "rectify_pair: two uint8 images of one size expected")
    H, W = L.shape
    ms = [np.ascontiguousarray(m, np.float32) for m in maps]
    if len(ms) != 4 or any(m.shape != (H, W) for m in ms):
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, "rectify_pair: four maps of the image size expected")
    x0, y0, x1, y1 = roi
    oL = np.empty((y1 - y0, x1 - x0), np.uint8)
    oR = np.empty_like(oL)
    arr = (ctypes.c_void_p * 4)(*[m.ctypes.data for m in ms])
    r = Rect(x0, y0, x1, y1)
    ctx = context(0)
    check(lib().mvsv_use_own_stream(ctx.handle), ctx.handle)
    check(lib().mvsv_rectify_pair(ctx.handle, L.ctypes.data, W, R.ctypes.data, W, W, H, arr,
                                  ctypes.byref(r), oL.ctypes.data, oL.shape[1], oR.ctypes.data,
                                  oR.shape[1]), ctx.handle)
    return oL, oR


def resize_size(width, height, fx, fy=None):
    """Output size of cv::resize(src, dst, Size(0, 0), fx, fy): (cvRound(w fx), cvRound(h fy))."""
    fy = fx if fy is None else fy
    w, h = ctypes.c_int(), ctypes.c_int()
    check(lib().mvsv_resize_size(int(width), int(height), float(fx), float(fy), ctypes.byref(w),
                                 ctypes.byref(h)))
    return w.value, h.value


def resize(src, fx, fy=None):
    """cv::resize(src, dst, Size(0, 0), fx, fy, INTER_LINEAR) of a uint8 image
    (OpenCV 3.4 fixed-point arithmetic, on the GPU).

    src: (H, W) uint8 numpy array (host path), or a (H, W) / (N, H, W) uint8
    torch tensor on a HIP device (device path, stream-ordered like compute()).
    """
    fy = fx if fy is None else fy
    if type(src).__module__.startswith("torch"):
        import torch
        if not (src.is_cuda and src.dtype == torch.uint8 and src.dim() in (2, 3)):
            raise MvsvError(_lib.MVSV_E_INVALID_ARG, "resize: uint8 device tensor expected")
        batched = src.dim() == 3
        s = src if batched else src.unsqueeze(0)
        if s.stride(2) != 1:
            s = s.contiguous()
        n, sh, sw = s.shape
        dw, dh = resize_size(sw, sh, fx, fy)
        out = torch.empty((n, dh, dw), dtype=torch.uint8, device=src.device)
        ctx = context(src.device.index or 0)
        check(lib().mvsv_set_stream(ctx.handle,
                                    ctypes.c_void_p(torch.cuda.current_stream(src.device).cuda_stream)),
              ctx.handle)
        check(lib().mvsv_resize_device(ctx.handle, n, s.data_ptr(), s.stride(1), s.stride(0), sw, sh,
                                       float(fx), float(fy), out.data_ptr(), dw, dh * dw), ctx.handle)
        return out if batched else out[0]
    a = np.ascontiguousarray(src, np.uint8)
    if a.ndim != 2:
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, "resize: a 2-D uint8 image expected")
    sh, sw = a.shape
    dw, dh = resize_size(sw, sh, fx, fy)
    out = np.empty((dh, dw), np.uint8)
    ctx = context(0)
    check(lib().mvsv_use_own_stream(ctx.handle), ctx.handle)
    check(lib().mvsv_resize(ctx.handle, a.ctypes.data, sw, sw, sh, float(fx), float(fy),
                            out.ctypes.data, dw), ctx.handle)
    return out
