"""StereoBM disparities-on-lanes kernel (bm_match2_kernel, mvsv_bm.hip) against
the oracle: every blockSize it covers (5..21) with numDisparities on both
sides of 64 (one wave per column group / two), forced tile heights, border
column groups on both sides, a frame batch through the device path, and the
general 16x16-tile kernel where the lanes kernel does not apply.
Reference: Disparity::bm (src/disparity.cpp:18-22) -> cv::StereoBM::compute."""
import numpy as np
import pytest

from tests.test_gpu_parity import bm_both, rand_pair, report

pytestmark = pytest.mark.gpu

GRID = [(bs, D) for bs in (5, 7, 9, 11, 13, 15, 17, 19, 21) for D in (16, 64, 80, 128)]


def rand_params(rng, bs, D):
    return dict(pre_filter_type=int(rng.choice([0, 1])), pre_filter_size=int(rng.choice([5, 9])),
                pre_filter_cap=int(rng.integers(1, 64)), block_size=bs,
                min_disparity=int(rng.integers(-8, 8)), num_disparities=D,
                texture_threshold=int(rng.choice([0, 10, 200])),
                uniqueness_ratio=int(rng.choice([0, 5, 15, 60])),
                speckle_window_size=0, speckle_range=0,
                disp12_max_diff=int(rng.choice([-1, 0, 2])))


@pytest.mark.parametrize("bs,D", GRID)
def test_bm_lanes_block_sizes(gpu, mvsv, oracle, bs, D):
    rng = np.random.default_rng(5000 + 131 * bs + D)
    # wide enough for interior and clamped column groups on both sides
    H, W = int(rng.integers(bs + 8, 96)), int(D + rng.integers(70, 200))
    p = rand_params(rng, bs, D)
    L, R = rand_pair(rng, H, W, int(rng.integers(0, min(D, 40))), int(rng.integers(0, 3)))
    got, want = bm_both(mvsv, oracle, L, R, p)
    assert np.array_equal(got, want), f"{p}: " + report(got, want)


@pytest.mark.parametrize("ty", [1, 4, 8, 24, 64])
def test_bm_lanes_tile_rows(gpu, mvsv, oracle, ty):
    """Forced tile heights (MVSV_OPT_BM_TILE_ROWS) give the same maps."""
    from mvstereovision3_amd import _lib
    rng = np.random.default_rng(6000 + ty)
    L, R = rand_pair(rng, 150, 260, 20, 1)
    try:
        for bs, D in ((9, 64), (21, 112)):
            p = rand_params(rng, bs, D)
            p.update(uniqueness_ratio=10, texture_threshold=10)
            _lib.set_option(_lib.OPT_BM_TILE_ROWS, ty)
            got, want = bm_both(mvsv, oracle, L, R, p)
            assert np.array_equal(got, want), f"TY={ty} {p}: " + report(got, want)
    finally:
        _lib.set_option(_lib.OPT_BM_TILE_ROWS, 0)


def test_bm_lanes_tile_rows_limits(gpu, mvsv, oracle):
    """The largest LDS image (128 rows, blockSize 21, D 128: ~158 KB of the
    160 KB) runs bit-exact; out-of-range option values are rejected."""
    from mvstereovision3_amd import _lib
    rng = np.random.default_rng(6500)
    L, R = rand_pair(rng, 200, 300, 30, 0)
    p = rand_params(rng, 21, 128)
    try:
        _lib.set_option(_lib.OPT_BM_TILE_ROWS, 128)
        got, want = bm_both(mvsv, oracle, L, R, p)
        assert np.array_equal(got, want), f"{p}: " + report(got, want)
        for bad in (-1, 129):
            with pytest.raises(_lib.MvsvError):
                _lib.set_option(_lib.OPT_BM_TILE_ROWS, bad)
    finally:
        _lib.set_option(_lib.OPT_BM_TILE_ROWS, 0)


def test_bm_lanes_batch_device(gpu, mvsv, oracle):
    """Three different frames in one device-path launch."""
    torch = gpu
    rng = np.random.default_rng(7000)
    H, W, D, bs = 120, 320, 96, 15
    p = rand_params(rng, bs, D)
    p.update(uniqueness_ratio=15, texture_threshold=10, disp12_max_diff=1)
    pairs = [rand_pair(rng, H, W, int(rng.integers(0, 40)), k % 3) for k in range(3)]
    m = mvsv.StereoBM.create(D, bs)
    for k, v in p.items():
        setattr(m._params, k, v)
    dev = torch.device("cuda", 0)
    Lb = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
    Rb = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
    out = torch.empty((3, H, W), dtype=torch.int16, device=dev)
    m.compute(Lb, Rb, out)
    got = out.cpu().numpy()
    for i, (L, R) in enumerate(pairs):
        want = oracle.bm(L, R, m.params())
        assert np.array_equal(got[i], want), f"frame {i}: " + report(got[i], want)


@pytest.mark.parametrize("bs,D", [(23, 32), (25, 144), (9, 160), (25, 160), (31, 256)])
def test_bm_general_kernel(gpu, mvsv, oracle, bs, D):
    """Shapes outside the lanes kernel (blockSize > 21 or D > 128) keep the
    16x16-tile kernel; (25, 160) and (31, 256) keep their window sums in a
    global scratch slab (the LDS image would exceed 160 KB)."""
    rng = np.random.default_rng(8000 + bs + D)
    H, W = 80, D + 150
    p = rand_params(rng, bs, D)
    p.update(pre_filter_type=1)
    L, R = rand_pair(rng, H, W, int(rng.integers(0, 30)), 1)
    got, want = bm_both(mvsv, oracle, L, R, p)
    assert np.array_equal(got, want), f"{p}: " + report(got, want)
