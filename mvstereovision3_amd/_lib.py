"""ctypes binding of libmvsv.so (the C ABI declared in include/mvsv.h).

The library is built in-tree by ``__graft_entry__.build()``
(mvstereovision3_amd/csrc/Makefile -> mvstereovision3_amd/libmvsv.so).  There
is no fallback: if the library is missing, every entry point raises
:class:`MvsvError`.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# MVSV_LIBRARY: an alternative in-tree build of the same ABI (A/B kernel variants)
LIB_PATH = os.environ.get("MVSV_LIBRARY") or os.path.join(_HERE, "libmvsv.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "mvsv.h")

MVSV_OK = 0
MVSV_E_INVALID_ARG = -1
MVSV_E_HIP = -2
MVSV_E_OOM = -3
MVSV_E_IO = -4
MVSV_E_PARSE = -5
MVSV_E_NODEV = -6
MVSV_E_TIMEOUT = -7

OPT_STRIP_SPIN_LIMIT = 1
OPT_BM_TILE_ROWS = 2
OPT_STRIP_WAVES = 3
OPT_PATH_SCHEDULE = 4
OPT_STRIP_TICKETS = 5
OPT_COST_RESIDUAL = 6
OPT_BITSLICE = 7

MODE_SGBM = 0
MODE_HH = 1
PREFILTER_NORMALIZED_RESPONSE = 0
PREFILTER_XSOBEL = 1
VARIANT_FIRSTCOL_FIX = 1
VARIANT_WTA_MIN_D = 2

NUM_STAGES = 9

_CODES = {
    MVSV_E_INVALID_ARG: "invalid argument",
    MVSV_E_HIP: "HIP error",
    MVSV_E_OOM: "out of memory",
    MVSV_E_IO: "cannot open file",
    MVSV_E_PARSE: "missing or malformed key",
    MVSV_E_NODEV: "no HIP device",
    MVSV_E_TIMEOUT: "strip hand-off gave up",
}


class MvsvError(RuntimeError):
    """Raised for every negative MVSV_E_* code (OpenCV would throw cv::Exception)."""

    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"mvsv error {code} ({_CODES.get(code, 'unknown')}){': ' + msg if msg else ''}")


SGBM_FIELDS = ("min_disparity", "num_disparities", "block_size", "p1", "p2",
               "disp12_max_diff", "pre_filter_cap", "uniqueness_ratio",
               "speckle_window_size", "speckle_range", "mode", "variant")
BM_FIELDS = ("pre_filter_type", "pre_filter_size", "pre_filter_cap", "block_size",
             "min_disparity", "num_disparities", "texture_threshold", "uniqueness_ratio",
             "speckle_window_size", "speckle_range", "disp12_max_diff")
YAML_FIELDS = ("minDisp", "numDisp", "blockSize", "disp12MaxDiff", "preFilterCap",
               "uniquenessRatio", "speckleWindowSize", "speckleRange", "disparityMode")


class SgbmParams(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int) for f in SGBM_FIELDS]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f in SGBM_FIELDS}


class BmParams(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int) for f in BM_FIELDS]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f in BM_FIELDS}


class Rect(ctypes.Structure):
    """mvsv_rect: half-open [x0, x1) x [y0, y1)."""
    _fields_ = [("x0", ctypes.c_int), ("y0", ctypes.c_int), ("x1", ctypes.c_int),
                ("y1", ctypes.c_int)]


class SgbmYamlValues(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int) for f in YAML_FIELDS]


_lib = None
_lock = threading.Lock()


def _declare(lib, strict=True):
    P = ctypes.c_void_p
    I = ctypes.c_int
    Z = ctypes.c_size_t
    sig = {
        "mvsv_version": ([], I),
        "mvsv_sgbm_params_default": ([P], None),
        "mvsv_sgbm_params_create": ([P] + [I] * 11, None),
        "mvsv_bm_params_default": ([P, I, I], None),
        "mvsv_sgbm_validate": ([P, I, I], I),
        "mvsv_bm_validate": ([P, I, I], I),
        "mvsv_create": ([ctypes.POINTER(P), I], I),
        "mvsv_destroy": ([P], None),
        "mvsv_last_error": ([P], ctypes.c_char_p),
        "mvsv_set_stream": ([P, P], I),
        "mvsv_use_own_stream": ([P], I),
        "mvsv_get_stream": ([P], P),
        "mvsv_synchronize": ([P], I),
        "mvsv_set_option": ([P, I, ctypes.c_longlong], I),
        "mvsv_trim": ([P], I),
        "mvsv_sgbm": ([P, P, Z, P, Z, I, I, P, P, Z], I),
        "mvsv_bm": ([P, P, Z, P, Z, I, I, P, P, Z], I),
        "mvsv_sgbm_device": ([P, I, P, Z, Z, P, Z, Z, I, I, P, P, Z, Z], I),
        "mvsv_bm_device": ([P, I, P, Z, Z, P, Z, Z, I, I, P, P, Z, Z], I),
        "mvsv_sgbm_workspace_bytes": ([I, I, I, P], Z),
        "mvsv_sgbm_plan": ([P, I, I, I, P, P], I),
        "mvsv_mean_disparity_grid_device": ([P, I, P, Z, Z, I, I, P], I),
        "mvsv_load_sgbm_yaml": ([ctypes.c_char_p, P, P], I),
        "mvsv_load_bm_yaml": ([ctypes.c_char_p, P], I),
        "mvsv_synth_pair": ([ctypes.c_uint32, I, I, I, I, P, P], I),
        "mvsv_profile_enable": ([P, I], I),
        "mvsv_profile_reset": ([P], I),
        "mvsv_profile_read": ([P, P, P, I], I),
        "mvsv_profile_stage_name": ([I], ctypes.c_char_p),
        "mvsv_mean_disparity_grid": ([P, P, Z, I, I, P], I),
        "mvsv_stream_create": ([P, I, I, P, I, P, ctypes.POINTER(P)], I),
        "mvsv_stream_set_params": ([P, P], I),
        "mvsv_stream_set_batch": ([P, I], I),
        "mvsv_stream_set_inflight": ([P, I], I),
        "mvsv_stream_push": ([P, P, Z, P, Z], I),
        "mvsv_stream_pop": ([P, P, Z, P], I),
        "mvsv_stream_pop_view": ([P, P, P], I),
        "mvsv_stream_pending": ([P], I),
        "mvsv_stream_destroy": ([P], None),
        "mvsv_remap_device": ([P, I, P, Z, Z, I, I, P, P, Z, P, Z, Z, I, I], I),
        "mvsv_rectify_pair": ([P, P, Z, P, Z, I, I, P, P, P, Z, P, Z], I),
        "mvsv_init_undistort_rectify_map": ([P, P, I, P, P, I, I, P, P, Z], I),
        "mvsv_resize_size": ([I, I, ctypes.c_double, ctypes.c_double, ctypes.POINTER(I),
                              ctypes.POINTER(I)], I),
        "mvsv_resize_device": ([P, I, P, Z, Z, I, I, ctypes.c_double, ctypes.c_double, P, Z, Z], I),
        "mvsv_resize": ([P, P, Z, I, I, ctypes.c_double, ctypes.c_double, P, Z], I),
        "mvsv_reproject_device": ([P, I, P, Z, Z, I, I, P, P, Z, Z], I),
        "mvsv_calc_coordinate": ([ctypes.c_float] * 3 + [P, P], None),
        "mvsv_calc_coordinates": ([ctypes.c_int, P, P, P], None),
        "mvsv_calc_distance": ([ctypes.c_float] * 3 + [P], ctypes.c_float),
        "mvsv_calc_dmap_values": ([P, P, P, P, P], None),
        "mvsv_write_ply": ([ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, P, Z, Z, I, P, Z,
                            I, I], I),
        "mvsv_dmap2pcl": ([P, ctypes.c_char_p, P, Z, I, I, P], I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name, None) if not strict else getattr(lib, name)
        if fn is None:  # older A/B builds (strict=False) may lack newer entry points
            continue
        fn.argtypes = args
        fn.restype = res
    return lib


def lib():
    """Load libmvsv.so (torch first, so both share one HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            try:  # torch bundles libamdhip64.so.7; load it first so the SONAME is shared
                import torch  # noqa: F401
            except ImportError:  # pragma: no cover - torch is always present in this image
                pass
            if not os.path.exists(LIB_PATH):
                raise MvsvError(MVSV_E_INVALID_ARG,
                                f"{LIB_PATH} is not built; run __graft_entry__.build()")
            _lib = _declare(ctypes.CDLL(LIB_PATH))
    return _lib


def check(rc: int, ctx=None) -> int:
    if rc < 0:
        msg = ""
        if ctx:
            raw = lib().mvsv_last_error(ctx)
            msg = raw.decode() if raw else ""
        raise MvsvError(rc, msg)
    return rc


class Context:
    """One mvsv_ctx (HIP stream + cached device buffers) per device and thread."""

    def __init__(self, device: int = 0):
        self.device = device
        h = ctypes.c_void_p()
        check(lib().mvsv_create(ctypes.byref(h), device))
        self.handle = h

    def close(self):
        if self.handle:
            lib().mvsv_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


class use_context:
    """``with use_context(ctx):`` -- this thread's calls on ``ctx.device`` run on
    ``ctx`` (its own stream-ordered buffers) instead of the thread's default
    context: independent batches then proceed concurrently on separate
    contexts / HIP streams (bench.py --inflight)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def __enter__(self):
        ov = getattr(_tls, "override", None)
        if ov is None:
            ov = _tls.override = {}
        self.prev = ov.get(self.ctx.device)
        ov[self.ctx.device] = self.ctx
        return self.ctx

    def __exit__(self, *exc):
        if self.prev is None:
            _tls.override.pop(self.ctx.device, None)
        else:
            _tls.override[self.ctx.device] = self.prev
        return False


def context(device: int = 0) -> Context:
    ov = getattr(_tls, "override", None)
    if ov and device in ov:
        return ov[device]
    ctxs = getattr(_tls, "ctxs", None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    c = ctxs.get(device)
    if c is None:
        c = ctxs[device] = Context(device)
    return c


def synchronize(device: int = 0) -> None:
    """Wait for the device work of this thread's context on `device` and raise
    MvsvError(MVSV_E_TIMEOUT) if an SGBM launch since the last check gave up a
    strip hand-off (its maps were written as all INVALID).  Call it where a
    torch.cuda.synchronize() would make the maps visible to the host."""
    c = context(device)
    check(lib().mvsv_synchronize(c.handle), c.handle)


def set_option(option: int, value: int, device: int = 0) -> None:
    c = context(device)
    check(lib().mvsv_set_option(c.handle, int(option), int(value)), c.handle)


def profile_enable(ctx: Context, on: bool = True):
    check(lib().mvsv_profile_enable(ctx.handle, 1 if on else 0), ctx.handle)


def profile_reset(ctx: Context):
    check(lib().mvsv_profile_reset(ctx.handle), ctx.handle)


def profile_read(ctx: Context) -> dict:
    """{stage_name: (total_ms, launches)} accumulated since the last reset."""
    ms = (ctypes.c_double * NUM_STAGES)()
    n = (ctypes.c_int * NUM_STAGES)()
    check(lib().mvsv_profile_read(ctx.handle, ms, n, NUM_STAGES), ctx.handle)
    return {lib().mvsv_profile_stage_name(i).decode(): (ms[i], n[i]) for i in range(NUM_STAGES)}


PLAN_BITSLICE, PLAN_SIDE, PLAN_STRIPS, PLAN_RESIDUAL = 1, 2, 4, 8


def sgbm_plan(ctx, n, width, height, params) -> int:
    """MVSV_PLAN_* bits of the pipeline ``ctx`` runs for an SGBM call of this
    shape (mvsv_sgbm_plan): bit-sliced, side by side / strips, residual plane."""
    out = ctypes.c_int(0)
    check(lib().mvsv_sgbm_plan(ctx.handle, n, width, height, ctypes.byref(params), ctypes.byref(out)), ctx.handle)
    return out.value
