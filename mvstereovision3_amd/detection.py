"""MeanDisparityDetection, Subimage and the camera-loop frame stream.

Mirrors src/MeanDisparityDetection.cpp:71-266, inc/Subimage.h:17-47,
trgt/mean_test.cpp:80-106 (createDMapROIS) and replaces the disparity worker
thread of trgt/mean_test.cpp:61-70 with DisparityStream (mvsv_stream_*: upload,
SGBM + 9x9 mean grid on the device, download, overlapped on HIP streams).
The 81 tile means are computed on the GPU (mean_grid_kernel); the 81-element
decisions stay on the host, exactly as the reference orders them.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref

import numpy as np

from . import _lib
from ._lib import MvsvError, Rect, check, context, lib
from .utility import PLY_WITH_COLOR, Utility, dMapValues, ply

MEAN_DISTANCE = 0
MEAN_VALUE = 1

# src/MeanDisparityDetection.cpp:21-66 (note: key 10 is absent, 81 is present)
POSITIONS = {}
_groups = ["TOP LEFT", "TOP", "TOP RIGHT", "LEFT", "CENTER", "RIGHT", "BOTTOM LEFT", "BOTTOM",
           "BOTTOM RIGHT"]
for _k in range(9):
    POSITIONS[_k] = f"TOP LEFT - {_k}"
POSITIONS.update({9: "TOP - 0"})
for _k in range(1, 9):
    POSITIONS[10 + _k] = f"TOP - {_k}"
for _g, _base in zip(_groups[2:], range(19, 82, 9)):
    for _k in range(9):
        POSITIONS[_base + _k] = f"{_g} - {_k}"


def create_dmap_rois(reference_shape, num_disp, binning=0, reload=False):
    """createDMapROIS (trgt/mean_test.cpp:80-106) -> (roi_u, roi_b) as (x0, y0, x1, y1)."""
    rows, cols = reference_shape
    shift = num_disp // 2
    if shift % 2 == 1:
        shift = shift + 1
        if (cols - shift) % 8 != 0:
            shift = shift + (cols - shift % 8)  # sic: operator precedence as in the reference
    roi_u = (shift, 0, cols, rows)
    roi_b = (shift // 2, 0, cols // 2, rows // 2)
    return roi_u, roi_b


class Subimage:
    """inc/Subimage.h: a tile with its centre and mean disparity value."""

    def __init__(self, tl=(0, 0), br=(0, 0)):
        self.tl = tuple(tl)
        self.br = tuple(br)
        tx, ty = br[0] - tl[0], br[1] - tl[1]
        self.roi_center = (tl[0] + int(tx / 2), tl[1] + int(ty / 2))
        self.value = 0.0

    def calculateSubimageValue(self, dMap):
        self.value = Utility.calcMeanDisparity(np.asarray(dMap)[self.tl[1]:self.br[1],
                                                                self.tl[0]:self.br[0]])


class MeanDisparityDetection:
    """src/MeanDisparityDetection.cpp with the 9x9 means computed on the GPU."""

    MEAN_DISTANCE = MEAN_DISTANCE
    MEAN_VALUE = MEAN_VALUE

    def __init__(self, pcl_dir="pcl/subimage_detection"):
        self.mSubimageVec: list[Subimage] = []
        self.mFoundObstacles: list[Subimage] = []
        self.mMeanMap: list[float] = []
        self.mMeanDistanceMap: list[float] = []
        self.mFoundPoints: list[np.ndarray] = []
        self.mObstacleCounter = 0
        self.mRange = (0.0, 0.0)
        self.mRangeDisparity = (0.0, 0.0)
        self.mDetectionMode = None
        self.mQ_32F = None
        self.mDMap = None
        self.pcl_dir = pcl_dir

    def init(self, reference, Q, min_distance, max_distance):
        """:71-112 — 9x9 tiles of (cols/9) x (rows/9) and the disparity range of [min, max] m."""
        shape = reference if isinstance(reference, tuple) else np.asarray(reference).shape
        rows, cols = shape[0], shape[1]
        self.mSubimageVec = []
        self.mQ_32F = np.asarray(Q, np.float32).reshape(4, 4)
        dx, dy = cols // 9, rows // 9
        for r in range(9):
            for c in range(9):
                tl = (c * dx, r * dy)
                br = (c * dx + dx, r * dy + dy)
                self.mSubimageVec.append(Subimage(tl, br))
                self.mFoundObstacles.append(Subimage(tl, br))
        # detectObstacles' batched coordinate call: tile centres and Q as float32
        self._centers = np.array([s.roi_center for s in self.mSubimageVec], np.float32).reshape(81, 2)
        self._q16 = np.ascontiguousarray(self.mQ_32F.reshape(16))
        lo = Utility.calcDMapValues([0, 0, np.float32(min_distance) * np.float32(1000)], self.mQ_32F)
        hi = Utility.calcDMapValues([0, 0, np.float32(max_distance) * np.float32(1000)], self.mQ_32F)
        self.mRangeDisparity = (lo.dValue, hi.dValue)

    def setRange(self, min_distance, max_distance):
        self.mRange = (float(np.float32(min_distance)), float(np.float32(max_distance)))

    def getRange(self):
        # ObstacleDetection::mRange is pair<float,float>; the derived getter returns pair<int,int>
        return int(self.mRange[0]), int(self.mRange[1])

    def getSubimageVec(self):
        return self.mSubimageVec

    def getMeanMap(self):
        return self.mMeanMap

    def getMeanDistanceMap(self):
        return self.mMeanDistanceMap

    def getFoundObstacles(self):
        return self.mFoundObstacles

    def getObstacleCounter(self):
        return self.mObstacleCounter

    def build(self, dMap, binning=0, mode=MEAN_VALUE, means=None):
        """:159-206.  dMap: host int16 map (or torch tensor on a HIP device).

        The tile means come from the GPU grid kernel (or `means`, e.g. from a
        DisparityStream pop).  MEAN_DISTANCE falls through into MEAN_VALUE, as the
        reference's switch does (no break), so the mode ends as MEAN_VALUE.
        """
        self.mDMap = dMap
        m = self._grid(dMap) if means is None else np.asarray(means, np.float32).reshape(81)
        if mode == MEAN_DISTANCE:
            self.mDetectionMode = MEAN_DISTANCE
            self.mMeanDistanceMap = []
            for i, s in enumerate(self.mSubimageVec):
                v = dMapValues(m[i], s.roi_center[0], s.roi_center[1])
                self.mMeanDistanceMap.append(Utility.calcDistance(v, self.mQ_32F, 0))
            mode = MEAN_VALUE
        if mode == MEAN_VALUE:
            self.mDetectionMode = MEAN_VALUE
            self.mMeanMap = m.tolist()
            for s, v in zip(self.mSubimageVec, self.mMeanMap):
                s.value = v

    def _grid(self, dMap):
        if type(dMap).__module__.startswith("torch"):
            from .disparity import mean_disparity_grid
            return mean_disparity_grid(dMap).cpu().numpy()
        d = np.asarray(dMap)
        if d.dtype != np.int16 or d.ndim != 2:
            raise MvsvError(_lib.MVSV_E_INVALID_ARG, "build: 2-D int16 map expected")
        if d.strides[1] != 2:
            d = np.ascontiguousarray(d)
        out = np.empty(81, np.float32)
        ctx = context(0)
        check(lib().mvsv_use_own_stream(ctx.handle), ctx.handle)
        check(lib().mvsv_mean_disparity_grid(ctx.handle, d.ctypes.data, d.strides[0] // 2,
                                             d.shape[1], d.shape[0], out.ctypes.data), ctx.handle)
        return out

    def detectObstacles(self, write_pcl=True):
        """:211-266.  Returns the list of position strings printed in MEAN_DISTANCE mode."""
        printed = []
        if self.mDetectionMode == MEAN_DISTANCE:
            for i, dist in enumerate(self.mMeanDistanceMap):
                if self.mRange[1] > dist > self.mRange[0]:
                    printed.append(POSITIONS.get(i, ""))
            return printed
        if self.mDetectionMode != MEAN_VALUE:
            return printed
        lo, hi = np.float32(self.mRangeDisparity[0]), np.float32(self.mRangeDisparity[1])
        # the reference's per-tile test (float32 compares) over all 81 means at
        # once, then every found tile's coordinate in one native call
        means = np.asarray(self.mMeanMap, np.float32)
        found = np.flatnonzero((means < lo) & (means > hi))
        self.mFoundObstacles = [self.mSubimageVec[i] for i in found]
        self.mFoundPoints = []
        if found.size:
            xyd = np.empty((found.size, 3), np.float32)
            xyd[:, 0] = self._centers[found, 0]
            xyd[:, 1] = self._centers[found, 1]
            xyd[:, 2] = means[found]
            pts = np.empty((found.size, 4), np.float32)
            lib().mvsv_calc_coordinates(int(found.size), xyd.ctypes.data, self._q16.ctypes.data, pts.ctypes.data)
            self.mFoundPoints = list(pts)
        if self.mFoundPoints and write_pcl:
            c = self.mObstacleCounter
            prefix = "000" if c < 10 else ("00" if c < 100 else "0")
            path = os.path.join(self.pcl_dir, f"pcl_{prefix}{c}.ply")
            dm = self.mDMap.cpu().numpy() if type(self.mDMap).__module__.startswith("torch") \
                else np.asarray(self.mDMap)
            ply("Hagen Hiller", "obstacle pointcloud", dm).write(path, np.stack(self.mFoundPoints),
                                                                 PLY_WITH_COLOR)
            self.mObstacleCounter += 1
        return printed


class DisparityStream:
    """Double-buffered camera-loop pipeline over mvsv_stream (include/mvsv.h).

    push(left, right) uploads a rectified pair and enqueues SGBM (+ the 9x9
    mean grid of grid_roi); pop() returns (disparity int16, means[81] or None)
    in push order.  `depth` frames may be in flight; with batch > 1 they are
    computed in groups of `batch` frames (frame-batch kernels); with inflight > 1
    up to that many groups run concurrently on the stream's compute lanes.
    """

    def __init__(self, matcher, width, height, depth=3, grid_roi=None, device=0, batch=1,
                 inflight=1):
        self._ctx = context(device)
        self.width, self.height = width, height
        self._params = matcher._params
        self._grid = grid_roi is not None
        roi = Rect(*grid_roi) if grid_roi is not None else None
        h = ctypes.c_void_p()
        check(lib().mvsv_stream_create(self._ctx.handle, width, height, ctypes.byref(self._params),
                                       depth, ctypes.byref(roi) if roi is not None else None,
                                       ctypes.byref(h)), self._ctx.handle)
        self._h = h
        # pinned host slots stay allocated while pop views are alive: a view's
        # buffer references the stream, and close() defers the destroy until
        # the last view is gone (use-after-free otherwise)
        self._live_views = 0
        self._close_pending = False
        # pop views are released by weakref finalizers, which may run from GC on
        # any thread: the view count, the pending close and the destroy share a lock
        self._views_lock = threading.RLock()
        if batch != 1:
            self.set_batch(batch)
        if inflight != 1:
            self.set_inflight(inflight)

    def set_inflight(self, n):
        """Up to n frame-batch launches in flight (mvsv_stream_set_inflight)."""
        check(lib().mvsv_stream_set_inflight(self._h, int(n)), self._ctx.handle)

    def set_batch(self, batch):
        """Compute frames `batch` at a time (mvsv_stream_set_batch)."""
        check(lib().mvsv_stream_set_batch(self._h, int(batch)), self._ctx.handle)

    def set_params(self, matcher):
        self._params = matcher._params
        check(lib().mvsv_stream_set_params(self._h, ctypes.byref(self._params)), self._ctx.handle)

    def pending(self):
        return int(lib().mvsv_stream_pending(self._h))

    def _live(self):
        if self.closed:
            raise MvsvError(_lib.MVSV_E_INVALID_ARG, "stream is closed")
        return self._h

    def push(self, left, right):
        self._live()
        L = np.asarray(left)
        R = np.asarray(right)
        if L.shape != (self.height, self.width) or R.shape != L.shape or L.dtype != np.uint8 \
                or R.dtype != np.uint8:
            raise MvsvError(_lib.MVSV_E_INVALID_ARG, "push: uint8 pair of the stream's size expected")
        if L.strides[1] != 1:
            L = np.ascontiguousarray(L)
        if R.strides[1] != 1:
            R = np.ascontiguousarray(R)
        check(lib().mvsv_stream_push(self._h, L.ctypes.data, L.strides[0], R.ctypes.data,
                                     R.strides[0]), self._ctx.handle)

    def pop(self, copy_map=True):
        """(map, means) of the oldest frame; copy_map=False returns (None, means);
        copy_map="view" returns a read-only view of the map in the stream's pinned
        host slot (no host copy), valid until the next push."""
        self._live()
        if copy_map == "view":
            ptr = ctypes.c_void_p()
            means = np.empty(81, np.float32) if self._grid else None
            check(lib().mvsv_stream_pop_view(self._h, ctypes.byref(ptr),
                                             means.ctypes.data if means is not None else None),
                  self._ctx.handle)
            buf = (ctypes.c_int16 * (self.width * self.height)).from_address(ptr.value)
            buf._owner = self  # numpy's base chain keeps the stream (and its slots) alive
            with self._views_lock:
                self._live_views += 1
            fin = weakref.finalize(buf, DisparityStream._view_released, self)
            fin.atexit = False  # no library calls during interpreter shutdown
            view = np.ctypeslib.as_array(buf).reshape(self.height, self.width)
            view.flags.writeable = False
            return view, means
        out = np.empty((self.height, self.width), np.int16) if copy_map else None
        means = np.empty(81, np.float32) if self._grid else None
        check(lib().mvsv_stream_pop(self._h, out.ctypes.data if out is not None else None, self.width,
                                    means.ctypes.data if means is not None else None),
              self._ctx.handle)
        return out, means

    @staticmethod
    def _view_released(stream):
        with stream._views_lock:
            stream._live_views -= 1
            if stream._close_pending and stream._live_views == 0:
                stream._destroy()

    def _destroy(self):
        with self._views_lock:
            if self._h:
                lib().mvsv_stream_destroy(self._h)
                self._h = None
            self._close_pending = False

    def close(self):
        """Destroys the stream; with pop views still alive, when the last one goes."""
        with self._views_lock:
            if self._live_views > 0:
                self._close_pending = True
                return
            self._destroy()

    @property
    def closed(self):
        return self._h is None or self._close_pending

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
