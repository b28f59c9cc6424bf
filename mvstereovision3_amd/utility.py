"""Host mirror of the reference's Utility:: reprojection helpers and ply writer.

Reference: src/utility.cpp:176-303 (calcCoordinate, calcDistance,
calcDMapValues, dmap2pcl, calcMeanDisparity, calcMinMaxDisparity) and
src/ply.cpp:37-133 (ply::write).  The per-pixel work (reproject) runs in the
HIP kernel behind mvsv_reproject_device; the single-point helpers and the PLY
text writer are host code in libmvsv.so (include/mvsv.h).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from ._lib import MvsvError, check, context, lib

PLY_PLAIN = 0
PLY_WITH_COLOR = 1
PLY_WITH_COLOR_SHADING = 2


def _q16(Q) -> np.ndarray:
    q = np.ascontiguousarray(np.asarray(Q, dtype=np.float32).reshape(16))
    return q


class dMapValues:  # noqa: N801 - reference name (inc/utility.h:50-55)
    def __init__(self, dValue=0.0, image_x=0.0, image_y=0.0):
        self.dValue = float(dValue)
        self.image_x = float(image_x)
        self.image_y = float(image_y)


class Utility:
    """Static mirror of namespace Utility (inc/utility.h:57-82)."""

    @staticmethod
    def calcCoordinate(v: dMapValues, Q) -> np.ndarray:
        """src/utility.cpp:176-198 -> float32 (X, Y, Z, 1)."""
        q = _q16(Q)
        out = np.empty(4, np.float32)
        lib().mvsv_calc_coordinate(v.image_x, v.image_y, v.dValue, q.ctypes.data, out.ctypes.data)
        return out

    @staticmethod
    def calcDistance(v: dMapValues, Q, binning: int = 0) -> float:
        """src/utility.cpp:200-222 (binning is unused, as in the reference)."""
        q = _q16(Q)
        return float(lib().mvsv_calc_distance(v.image_x, v.image_y, v.dValue, q.ctypes.data))

    @staticmethod
    def calcDMapValues(c, Q) -> dMapValues:
        """src/utility.cpp:224-240: metric (x, y, z) -> image position and disparity * 16."""
        q = _q16(Q)
        c3 = np.ascontiguousarray(np.asarray(c, np.float32).reshape(-1)[:3])
        x = ctypes.c_float()
        y = ctypes.c_float()
        d = ctypes.c_float()
        lib().mvsv_calc_dmap_values(c3.ctypes.data, q.ctypes.data, ctypes.byref(x), ctypes.byref(y),
                                    ctypes.byref(d))
        return dMapValues(d.value, x.value, y.value)

    @staticmethod
    def dmap2pcl(filename: str, dMap, Q) -> None:
        """src/utility.cpp:242-262: PLY of every pixel with disparity > 0 (WITH_COLOR)."""
        d = np.asarray(dMap)
        if d.ndim != 2 or d.dtype != np.int16:
            raise MvsvError(_lib.MVSV_E_INVALID_ARG, "dmap2pcl: 2-D int16 map expected")
        if d.strides[1] != 2:
            d = np.ascontiguousarray(d)
        q = _q16(Q)
        ctx = context(0)
        check(lib().mvsv_use_own_stream(ctx.handle), ctx.handle)
        check(lib().mvsv_dmap2pcl(ctx.handle, os.fsencode(filename), d.ctypes.data, d.strides[0] // 2,
                                  d.shape[1], d.shape[0], q.ctypes.data), ctx.handle)

    @staticmethod
    def calcMeanDisparity(matrix) -> float:
        """src/utility.cpp:265-285: integer mean of values > 1 (0 when none)."""
        m = np.asarray(matrix).astype(np.int64)
        v = m[m > 1]
        if v.size == 0 or int(v.sum()) == 0:
            return 0.0
        t, n = int(v.sum()), int(v.size)
        q = abs(t) // n * (1 if t >= 0 else -1)  # C++ int division truncates toward 0
        return float(np.float32(q))

    @staticmethod
    def calcMinMaxDisparity(matrix):
        """src/utility.cpp:286-303: min / max of the positive values."""
        m = np.asarray(matrix)
        v = m[m > 0]
        if v.size == 0:
            raise MvsvError(_lib.MVSV_E_INVALID_ARG, "calcMinMaxDisparity: no positive value")
        return int(v.min()), int(v.max())


def reproject(dmap, Q):
    """Utility::calcCoordinate for every pixel of an int16 device map, on the GPU.

    dmap: (H, W) or (N, H, W) int16 torch tensor on a HIP device.  Returns a
    float32 tensor (..., H, W, 4) = (X, Y, Z, valid) with valid = (d > 0).
    """
    import torch
    if not (type(dmap).__module__.startswith("torch") and dmap.is_cuda and dmap.dtype == torch.int16):
        raise MvsvError(_lib.MVSV_E_INVALID_ARG, "reproject: int16 device tensor expected")
    batched = dmap.dim() == 3
    d = dmap if batched else dmap.unsqueeze(0)
    if d.stride(2) != 1:
        d = d.contiguous()
    n, H, W = d.shape
    out = torch.empty((n, H, W, 4), dtype=torch.float32, device=dmap.device)
    q = _q16(Q)
    ctx = context(dmap.device.index or 0)
    check(lib().mvsv_set_stream(ctx.handle,
                                ctypes.c_void_p(torch.cuda.current_stream(dmap.device).cuda_stream)),
          ctx.handle)
    check(lib().mvsv_reproject_device(ctx.handle, n, d.data_ptr(), d.stride(1), d.stride(0), W, H,
                                      q.ctypes.data, out.data_ptr(), W, H * W), ctx.handle)
    return out if batched else out[0]


class ply:  # noqa: N801 - reference name (inc/ply.h)
    """src/ply.cpp: ASCII PLY writer with the reference's three modes."""

    PLAIN = PLY_PLAIN
    WITH_COLOR = PLY_WITH_COLOR
    WITH_COLOR_SHADING = PLY_WITH_COLOR_SHADING

    def __init__(self, author: str = "", object_name: str = "", disparity_map=None):
        self.mAuthor = author
        self.mObjectName = object_name
        self.mDMap = None if disparity_map is None else np.asarray(disparity_map)

    def write(self, filename: str, to_write, mode: int) -> bool:
        """ply::write: to_write = sequence of (x, y, z[, ...]) points."""
        pts = np.ascontiguousarray(np.asarray(to_write, np.float32).reshape(len(to_write), -1))
        if pts.size and pts.shape[1] < 3:
            raise MvsvError(_lib.MVSV_E_INVALID_ARG, "ply.write: 3 coordinates per vertex")
        stride = pts.shape[1] if pts.size else 3
        d = self.mDMap
        if mode != PLY_PLAIN and (d is None or d.size == 0):
            return False  # "if(mDMap.rows == 0 || mDMap.cols == 0) return false;"
        dp, ds, W, H = None, 0, 0, 0
        if d is not None and d.size:
            d = np.ascontiguousarray(d.astype(np.int16, copy=False))
            dp, ds, W, H = d.ctypes.data, d.strides[0] // 2, d.shape[1], d.shape[0]
        rc = lib().mvsv_write_ply(os.fsencode(filename), self.mAuthor.encode(),
                                  self.mObjectName.encode(), pts.ctypes.data if pts.size else None,
                                  len(pts), stride, mode, dp, ds, W, H)
        if rc == _lib.MVSV_E_INVALID_ARG and mode != PLY_PLAIN:
            raise MvsvError(rc, "ply.write: the disparity map has no positive value")
        check(rc)
        return True
