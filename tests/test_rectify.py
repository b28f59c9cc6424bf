"""Rectification: oracle known answers and map construction.

The remap oracle restates OpenCV 3.4's RemapInvoker + remapBilinear fixed-point
path (oracle/mvsv_oracle.c: orc_remap_linear); parity unpinned (OpenCV absent).
The GPU kernel is compared with it bit-exactly in test_gpu_parity.py.
"""
import numpy as np


def test_remap_identity_and_integer_shift(oracle):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (40, 60)).astype(np.uint8)
    yy, xx = np.mgrid[0:40, 0:60].astype(np.float32)
    assert np.array_equal(oracle.remap_linear(img, xx, yy), img)
    out = oracle.remap_linear(img, xx + 3, yy - 2)
    assert np.array_equal(out[2:, :-3], img[:-2, 3:])
    # footprints (partially) outside read 0 (BORDER_CONSTANT; integer shift -> zero weights inside)
    assert not out[:2, :].any() and not out[:, 57:].any()


def test_remap_half_pixel_rounding(oracle):
    img = np.array([[10, 21, 0, 255]], np.uint8)
    mx = np.array([[0.5, 1.5, 2.5, 0.25]], np.float32)
    my = np.zeros_like(mx)
    got = oracle.remap_linear(img, mx, my)
    # weights 16/16 of 32: (10*16 + 21*16)*32 = 15872 -> (15872 + 16384) >> 15 = 0?  compute exactly
    def ref(a, b, ax):
        return ((a * (32 - ax) * 32 * 32 + b * ax * 32 * 32) + (1 << 14)) >> 15
    assert got[0, 0] == ref(10, 21, 16) and got[0, 1] == ref(21, 0, 16)
    assert got[0, 2] == ref(0, 255, 16) and got[0, 3] == ref(10, 21, 8)


def test_remap_round_half_even_map_conversion(oracle):
    # X = cvRound(x * 32): 1/64 * 32 = 0.5 -> 0 (even), 3/64 * 32 = 1.5 -> 2
    img = np.array([[0, 64]], np.uint8)
    got = oracle.remap_linear(img, np.array([[1 / 64, 3 / 64]], np.float32), np.zeros((1, 2), np.float32))
    assert got[0, 0] == 0 and got[0, 1] == ((64 * 2 * 32 * 32) + (1 << 14)) >> 15


def test_init_undistort_rectify_map_identity_and_distortion(mvsv):
    K = np.array([[300.0, 0, 160], [0, 300.0, 120], [0, 0, 1]])
    mx, my = mvsv.init_undistort_rectify_map(K, None, np.eye(3), K, (320, 240))
    yy, xx = np.mgrid[0:240, 0:320]
    assert np.allclose(mx, xx, atol=1e-4) and np.allclose(my, yy, atol=1e-4)
    d = [-0.2, 0.05, 0.001, -0.002, 0.01]
    mx2, my2 = mvsv.init_undistort_rectify_map(K, d, np.eye(3), K, (320, 240))
    # restate the OpenCV model in numpy double precision
    x = (xx - 160) / 300.0
    y = (yy - 120) / 300.0
    r2 = x * x + y * y
    kr = 1 + ((d[4] * r2 + d[1]) * r2 + d[0]) * r2
    u = 300 * (x * kr + d[2] * 2 * x * y + d[3] * (r2 + 2 * x * x)) + 160
    v = 300 * (y * kr + d[2] * (r2 + 2 * y * y) + d[3] * 2 * x * y) + 120
    assert np.allclose(mx2, u.astype(np.float32), atol=2e-3) and np.allclose(my2, v.astype(np.float32), atol=2e-3)
