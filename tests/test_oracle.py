"""CPU oracle checks (no GPU): golden fixtures, the two-restatement cross-check
and known-answer tests.  The oracle restates OpenCV 3.4 (third-party, absent
here): parity is unpinned, so agreement between the loop-structured C oracle
and the closed-form numpy twin is the transcription check.
"""
import json
import os

import numpy as np
import pytest

from tests.conftest import GOLDEN

FIX = np.load(os.path.join(GOLDEN, "fixtures.npz"))
META = json.load(open(os.path.join(GOLDEN, "fixtures.json")))


@pytest.mark.parametrize("case", META["sgbm"], ids=lambda c: c["name"])
def test_sgbm_fixtures(oracle, case):
    n = case["name"]
    got = oracle.sgbm(FIX[n + "_L"], FIX[n + "_R"], case["params"], flags=case["variant"])
    assert np.array_equal(got, FIX[n + "_out"])


@pytest.mark.parametrize("case", META["bm"], ids=lambda c: c["name"])
def test_bm_fixtures(oracle, case):
    n = case["name"]
    got = oracle.bm(FIX[n + "_L"], FIX[n + "_R"], case["params"])
    assert np.array_equal(got, FIX[n + "_out"])


def test_twin_reproduces_fixtures():
    from oracle import twin
    for case in META["sgbm"][:3]:
        n = case["name"]
        got = twin.sgbm_compute(FIX[n + "_L"], FIX[n + "_R"], case["params"], case["variant"])
        assert np.array_equal(got, FIX[n + "_out"]), n
    for case in META["bm"]:
        n = case["name"]
        assert np.array_equal(twin.bm_compute(FIX[n + "_L"], FIX[n + "_R"], case["params"]),
                              FIX[n + "_out"]), n


def test_cost_volume_fixture(oracle):
    from oracle import twin
    p = META["costvol_params"]
    C = oracle.sgbm_cost_volume(FIX["costvol_L"], FIX["costvol_R"], p)
    assert np.array_equal(C, FIX["costvol_C"])
    assert np.array_equal(twin.sgbm_cost_volume(FIX["costvol_L"], FIX["costvol_R"], p),
                          FIX["costvol_C"])


def test_post_fixtures(oracle):
    d = FIX["post_in"]
    assert np.array_equal(oracle.median3x3(d), FIX["post_median"])
    assert np.array_equal(oracle.filter_speckles(d, 0, 20, 16), FIX["post_speckle"])
    assert np.array_equal(oracle.mean_disparity_grid(d), FIX["post_grid"])


def _rand_pair(rng, H, W, shift, kind):
    if kind == 0:
        from scipy.ndimage import uniform_filter
        L = uniform_filter(rng.integers(0, 256, (H, W)).astype(float), 3).round().astype(np.uint8)
    elif kind == 1:
        L = (rng.integers(0, 4, (H, W)) * 60).astype(np.uint8)
        L[:, W // 3:W // 2] = 128
    else:
        L = rng.integers(0, 256, (H, W)).astype(np.uint8)
    R = np.roll(L, -shift, axis=1)
    R = np.clip(R.astype(int) + rng.integers(-2, 3, R.shape), 0, 255).astype(np.uint8)
    return L, R


@pytest.mark.parametrize("seed", range(12))
def test_cross_check_sgbm(oracle, seed):
    from oracle import twin
    rng = np.random.default_rng(seed)
    H, W = int(rng.integers(12, 40)), int(rng.integers(40, 80))
    D = int(rng.choice([16, 32]))
    p = dict(min_disparity=int(rng.integers(-5, 5)), num_disparities=D,
             block_size=int(rng.choice([0, 1, 3, 5, 7, 9])),
             p1=int(rng.choice([0, 2, 72, 300])), p2=int(rng.choice([0, 5, 288, 4000])),
             disp12_max_diff=int(rng.integers(-1, 4)),
             pre_filter_cap=int(rng.choice([0, 15, 31, 63])),
             uniqueness_ratio=int(rng.choice([-1, 0, 5, 15])),
             speckle_window_size=int(rng.choice([0, 10, 50])),
             speckle_range=int(rng.choice([1, 2, 4])), mode=int(rng.integers(0, 2)))
    if W + min(p["min_disparity"], 0) - max(p["min_disparity"] + D, 0) <= 5:
        p["num_disparities"] = 16
    L, R = _rand_pair(rng, H, W, int(rng.integers(0, 16)), int(rng.integers(0, 3)))
    flags = int(rng.integers(0, 4))
    assert np.array_equal(oracle.sgbm(L, R, p, flags), twin.sgbm_compute(L, R, p, flags))


@pytest.mark.parametrize("seed", range(12))
def test_cross_check_bm(oracle, seed):
    from oracle import twin
    rng = np.random.default_rng(100 + seed)
    H, W = int(rng.integers(24, 60)), int(rng.integers(60, 110))
    bs = int(rng.choice([5, 7, 9, 11, 21]))
    if bs >= min(H, W):
        bs = 5
    p = dict(pre_filter_type=1, pre_filter_size=9, pre_filter_cap=int(rng.integers(1, 64)),
             block_size=bs, min_disparity=int(rng.integers(-4, 4)),
             num_disparities=int(rng.choice([16, 32])),
             texture_threshold=int(rng.choice([0, 10, 100])),
             uniqueness_ratio=int(rng.choice([0, 10, 15])),
             speckle_window_size=int(rng.choice([0, 10])), speckle_range=int(rng.choice([0, 4, 32])),
             disp12_max_diff=int(rng.choice([-1, 0, 1, 3])))
    L, R = _rand_pair(rng, H, W, int(rng.integers(0, 16)), int(rng.integers(0, 3)))
    assert np.array_equal(oracle.bm(L, R, p), twin.bm_compute(L, R, p))


# ------------------------------------------------------ known answers -----
def _random_dot(H, W, shift, seed=7):
    rng = np.random.default_rng(seed)
    L = rng.integers(0, 256, (H, W)).astype(np.uint8)
    R = np.zeros_like(L)
    R[:, : W - shift] = L[:, shift:]
    R[:, W - shift:] = rng.integers(0, 256, (H, shift))
    return L, R


@pytest.mark.parametrize("mode", [0, 1])
def test_known_answer_sgbm_constant_shift(oracle, mode):
    d_true = 7
    L, R = _random_dot(48, 96, d_true)
    p = dict(min_disparity=0, num_disparities=16, block_size=5, p1=200, p2=800, disp12_max_diff=1,
             pre_filter_cap=31, uniqueness_ratio=10, speckle_window_size=0, speckle_range=0,
             mode=mode)
    d = oracle.sgbm(L, R, p)
    inner = d[8:-8, 24:-8]
    assert ((inner.astype(int) + 8) >> 4 == d_true).mean() > 0.99


def test_known_answer_bm_constant_shift(oracle):
    d_true = 11
    L, R = _random_dot(64, 128, d_true)
    p = dict(pre_filter_type=1, pre_filter_size=9, pre_filter_cap=31, block_size=9,
             min_disparity=0, num_disparities=32, texture_threshold=10, uniqueness_ratio=15,
             speckle_window_size=0, speckle_range=0, disp12_max_diff=-1)
    d = oracle.bm(L, R, p)
    inner = d[8:-8, 40:-8]
    assert ((inner.astype(int) + 8) >> 4 == d_true).mean() > 0.99


def test_constant_image_bm_all_filtered(oracle):
    L = np.full((40, 80), 100, np.uint8)
    p = dict(pre_filter_type=1, pre_filter_size=9, pre_filter_cap=31, block_size=9,
             min_disparity=0, num_disparities=16, texture_threshold=10, uniqueness_ratio=15,
             speckle_window_size=0, speckle_range=0, disp12_max_diff=-1)
    assert (oracle.bm(L, L, p) == -16).all()


def test_sgbm_no_columns_all_invalid(oracle):
    L = np.zeros((20, 40), np.uint8)
    p = dict(min_disparity=2, num_disparities=48, block_size=5, p1=0, p2=0, disp12_max_diff=0,
             pre_filter_cap=0, uniqueness_ratio=0, speckle_window_size=0, speckle_range=0, mode=0)
    assert (oracle.sgbm(L, L, p) == 16).all()  # INVALID = (minD - 1) * 16


def test_sgbm_saturated_costs_invalid(oracle):
    """All S saturate at MAX_COST -> no strict minimum -> bestDisp = -1 -> INVALID."""
    from oracle import twin
    rng = np.random.default_rng(3)
    L = rng.integers(0, 256, (16, 77)).astype(np.uint8)
    R = np.roll(L, -5, axis=1)
    p = dict(min_disparity=-4, num_disparities=16, block_size=11, p1=0, p2=4000,
             disp12_max_diff=-1, pre_filter_cap=63, uniqueness_ratio=0, speckle_window_size=0,
             speckle_range=1, mode=1)
    a = oracle.sgbm(L, R, p, core_only=True)
    assert np.array_equal(a, twin.sgbm_core(L, R, p))
    assert (a == -80).any()


def test_oracle_resize_linear_properties(oracle):
    """orc_resize_linear (cv::resize INTER_LINEAR restatement): factor 1 is the
    identity, a factor of 0.5 is the rounded 2x2 mean on whole blocks, and every
    output lies within one grey level of exact bilinear interpolation (OpenCV's
    pixel-centre convention, x clamped) -- the fixed-point rounding is the only
    difference.  Parity of the rounding itself is unpinned (OpenCV absent)."""
    rs = np.random.RandomState(3)
    a = rs.randint(0, 256, (37, 53)).astype(np.uint8)
    assert np.array_equal(oracle.resize_linear(a, 1.0, 1.0), a)
    # a factor that rounds back to the input size is a plain copy in OpenCV 3.4
    # (resize: dsize == ssize -> src.copyTo(dst)), not a resampling
    b = rs.randint(0, 256, (600, 600)).astype(np.uint8)
    assert np.array_equal(oracle.resize_linear(b, 1.0005, 0.9995), b)
    h = oracle.resize_linear(a, 0.5, 0.5)
    assert h.shape == (18, 26)  # cvRound(18.5) = 18, cvRound(26.5) = 26 (half to even)
    q = a[:36, :52].astype(int)
    blk = (q[0::2, 0::2] + q[1::2, 0::2] + q[0::2, 1::2] + q[1::2, 1::2] + 2) >> 2
    assert np.array_equal(h, blk)
    for f in (0.75, 1.5, 0.37, 2.0):
        r = oracle.resize_linear(a, f, f).astype(float)
        dh, dw = r.shape
        xs = np.clip((np.arange(dw) + 0.5) / f - 0.5, 0, 52)
        ys = np.clip((np.arange(dh) + 0.5) / f - 0.5, 0, 36)
        x0, y0 = np.floor(xs).astype(int), np.floor(ys).astype(int)
        x1, y1 = np.minimum(x0 + 1, 52), np.minimum(y0 + 1, 36)
        ax, ay = xs - x0, (ys - y0)[:, None]
        A = a.astype(float)
        ref = (A[y0][:, x0] * (1 - ax) + A[y0][:, x1] * ax) * (1 - ay) + \
              (A[y1][:, x0] * (1 - ax) + A[y1][:, x1] * ax) * ay
        assert np.abs(r - ref).max() <= 1.0, f


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_cost_residual_invariance(seed):
    """The cost residual plane (mvsv.h MVSV_OPT_COST_RESIDUAL) on the numpy twin:
    with R = min(C - min_d C, 2*P2) + P2 every direction's path deltas
    L_r - (C - P2) equal those computed from C, and the aggregated
    S'' = n*(R - P2) + deltas has the argmin (first minimum) of S and the same
    minimum up to n*(min_d C - P2) -- the identity the direction kernels and
    the residual final kernel rely on (no-wrap regime, 3*P2 <= 15)."""
    from oracle import twin
    rng = np.random.default_rng(700 + seed)
    H, W, D = 24, 70, 16
    L = rng.integers(0, 256, (H, W)).astype(np.uint8)
    L[:, 20:30] = 90  # flat patch: ties and equal costs
    R = np.roll(L, -3, axis=1).astype(int) + rng.integers(-2, 3, (H, W))
    R = np.clip(R, 0, 255).astype(np.uint8)
    p = dict(min_disparity=0, num_disparities=D, block_size=3, p1=2, p2=5, disp12_max_diff=1,
             pre_filter_cap=0, uniqueness_ratio=0, speckle_window_size=0, speckle_range=0,
             mode=seed % 2)
    e = twin.sgbm_effective(p, W)
    P1, P2 = e["P1"], e["P2"]
    C = twin.sgbm_cost_volume(L, R, p).astype(np.int32)
    m = C.min(axis=-1, keepdims=True)
    Rr = np.minimum(C - m, 2 * P2) + P2
    Ssum = np.zeros_like(C)
    Spp = np.zeros_like(C)
    dirs = twin.sgbm_directions(p["mode"])
    for dx, dy in dirs:
        dC = twin.sgbm_path(C, dx, dy, P1, P2) - (C - P2)
        dR = twin.sgbm_path(Rr, dx, dy, P1, P2) - (Rr - P2)
        assert np.array_equal(dC, dR), (dx, dy)
        assert dC.min() >= 0 and dC.max() <= P2
        Ssum += dC
        Spp += dR
    n = len(dirs)
    S = n * (C - P2) + Ssum       # no saturation at these sizes
    S2 = n * (Rr - P2) + Spp
    assert np.array_equal(S.argmin(axis=-1), S2.argmin(axis=-1))
    assert np.array_equal(S.min(axis=-1), S2.min(axis=-1) + n * (m[..., 0] - P2))


@pytest.mark.parametrize("cap", [15, 63])
def test_fullrate_bounds_of_the_cost_sums(cap):
    """The bounds behind the cost kernel's full-rate 32-bit sums and the BT
    distance rewrite, on the numpy twin with adversarial input
    (alternating 0 / 255 columns and rows: the largest Sobel and raw-channel
    intervals): every pixel cost <= 2*ftzero + 255 // 4 <= 189, so a 15x15 window sum
    stays < 2^16; and max(u - v1, v0 - u, 0) == sat(u - v1) + sat(v0 - u) for
    every interval (v0 <= v1)."""
    from oracle import twin
    rng = np.random.default_rng(cap)
    H, W, D = 20, 90, 32
    L = np.where((np.arange(W)[None, :] + np.arange(H)[:, None]) % 2, 255, 0).astype(np.uint8)
    R = np.where(rng.random((H, W)) < 0.5, 255, 0).astype(np.uint8)
    p = dict(min_disparity=0, num_disparities=D, block_size=3, p1=2, p2=5, disp12_max_diff=1,
             pre_filter_cap=cap, uniqueness_ratio=0, speckle_window_size=0, speckle_range=0, mode=1)
    e = twin.sgbm_effective(p, W)
    pix = twin.sgbm_pixel_cost(L, R, e)
    assert pix.max() <= 2 * e["ftzero"] + 255 // 4 <= 189
    assert 15 * 15 * 189 < 1 << 16
    # the interval-distance identity on every (u, [v0, v1]) of bytes
    u = np.arange(256, dtype=np.int16)[:, None, None]
    v0 = np.arange(256, dtype=np.int16)[None, :, None]
    v1 = np.arange(256, dtype=np.int16)[None, None, :]
    ok = v0 <= v1
    lhs = np.maximum(np.maximum(u - v1, v0 - u), 0)
    rhs = np.maximum(u - v1, 0) + np.maximum(v0 - u, 0)
    assert np.array_equal(np.where(ok, lhs, 0), np.where(ok, rhs, 0))
