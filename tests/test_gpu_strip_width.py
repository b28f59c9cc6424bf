"""Strip width of the SGBM sheared-strip path kernel (sgbm_tri_kernel, WV
compute waves per strip): the narrow shape (latency, chosen for one or two
frames) and the wide shape (throughput, chosen for frame batches) forced on the
same inputs, both bit-exact against the oracle -- D = 32..128 (8 / 15 waves)
and D = 256 (4 / 7 waves), 5 and 8 paths, the no-wrap and the general
recurrence, a frame batch through the device path.
Reference: Disparity::sgbm (src/disparity.cpp:6-10) -> cv::StereoSGBM::compute."""
import numpy as np
import pytest

from tests.test_gpu_parity import rand_pair, report, sgbm_both

pytestmark = pytest.mark.gpu

CASES = [
    # (H, W, D, blockSize, P1, P2, mode)
    (61, 200, 64, 5, 8, 32, 1),      # no-wrap, 8 paths
    (47, 170, 32, 3, 2, 5, 0),       # 5 paths
    (90, 300, 128, 9, 72, 288, 1),   # sgbm.yml-like P1/P2
    (40, 160, 64, 11, 300, 4000, 1),  # general (wrapping) recurrence
    (33, 420, 256, 3, 8, 96, 1),     # D = 256: wide = 7 waves
]


@pytest.mark.parametrize("shape", ["narrow", "wide"])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_strip_width_forced(gpu, mvsv, oracle, case, shape):
    from mvstereovision3_amd import _lib
    H, W, D, bs, P1, P2, mode = CASES[case]
    waves = {("narrow", False): 8, ("narrow", True): 4, ("wide", False): 15, ("wide", True): 7}[(shape, D > 128)]
    rng = np.random.default_rng(9100 + 7 * case)
    L, R = rand_pair(rng, H, W, int(rng.integers(0, min(D, 48))), int(rng.integers(0, 3)))
    kw = dict(minDisparity=int(rng.integers(-3, 3)), numDisparities=D, blockSize=bs, P1=P1, P2=P2,
              disp12MaxDiff=1, uniquenessRatio=10, mode=mode)
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 1)  # strips (small launches would run directions side by side)
        _lib.set_option(_lib.OPT_STRIP_WAVES, waves)
        got, want = sgbm_both(mvsv, oracle, L, R, **kw)
    finally:
        _lib.set_option(_lib.OPT_STRIP_WAVES, 0)
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    assert np.array_equal(got, want), f"waves={waves} {kw}: " + report(got, want)


def test_strip_width_batch_device(gpu, mvsv, oracle):
    """Three frames in one launch with narrow strips forced (the automatic
    choice for small launches is narrow; wide is covered by the 1280x960
    batch tests)."""
    from mvstereovision3_amd import _lib
    torch = gpu
    rng = np.random.default_rng(9200)
    H, W, D = 96, 260, 64
    pairs = [rand_pair(rng, H, W, int(rng.integers(0, 40)), k % 3) for k in range(3)]
    m = mvsv.StereoSGBM.create(minDisparity=1, numDisparities=D, blockSize=7, P1=8, P2=40,
                               disp12MaxDiff=1, uniquenessRatio=5, mode=1)
    dev = torch.device("cuda", 0)
    Lb = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
    Rb = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
    out = torch.empty((3, H, W), dtype=torch.int16, device=dev)
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 1)
        _lib.set_option(_lib.OPT_STRIP_WAVES, 8)
        m.compute(Lb, Rb, out)
        got = out.cpu().numpy()
    finally:
        _lib.set_option(_lib.OPT_STRIP_WAVES, 0)
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    p = dict(min_disparity=1, num_disparities=D, block_size=7, p1=8, p2=40, disp12_max_diff=1,
             pre_filter_cap=0, uniqueness_ratio=5, speckle_window_size=0, speckle_range=0, mode=1)
    for i, (L, R) in enumerate(pairs):
        want = oracle.sgbm(L, R, p)
        assert np.array_equal(got[i], want), f"frame {i}: " + report(got[i], want)


@pytest.mark.parametrize("tickets", [1, 0])
def test_strip_order_batch_device(gpu, mvsv, oracle, tickets):
    """Strips by ticket drawn on arrival (default for launches of more blocks
    than CUs: no dispatch-order assumption) and by blockIdx: both bit-exact on
    an 8-frame wide-strip batch of 304 blocks (> 256 CUs), twice in a row (the
    ticket counter carries over between launches)."""
    from mvstereovision3_amd import _lib
    torch = gpu
    rng = np.random.default_rng(9300)
    H, W, D, N = 300, 900, 64, 8  # 19 strips x 8 frames x 2 passes = 304 blocks
    pairs = [rand_pair(rng, H, W, int(rng.integers(0, 40)), k % 3) for k in range(N)]
    m = mvsv.StereoSGBM.create(minDisparity=0, numDisparities=D, blockSize=5, P1=8, P2=32,
                               disp12MaxDiff=1, uniquenessRatio=10, mode=1)
    dev = torch.device("cuda", 0)
    Lb = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
    Rb = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
    out = torch.empty((N, H, W), dtype=torch.int16, device=dev)
    outs = []
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 1)
        _lib.set_option(_lib.OPT_STRIP_WAVES, 15)
        _lib.set_option(_lib.OPT_STRIP_TICKETS, tickets)
        for _ in range(2):
            m.compute(Lb, Rb, out)
            outs.append(out.cpu().numpy())
    finally:
        _lib.set_option(_lib.OPT_STRIP_TICKETS, 1)
        _lib.set_option(_lib.OPT_STRIP_WAVES, 0)
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    p = dict(min_disparity=0, num_disparities=D, block_size=5, p1=8, p2=32, disp12_max_diff=1,
             pre_filter_cap=0, uniqueness_ratio=10, speckle_window_size=0, speckle_range=0, mode=1)
    for i, (L, R) in enumerate(pairs):
        want = oracle.sgbm(L, R, p)
        for got in outs:
            assert np.array_equal(got[i], want), f"tickets={tickets} frame {i}: " + report(got[i], want)


@pytest.mark.parametrize("tickets", [1, 0])
def test_strip_order_one_frame_resident(gpu, mvsv, oracle, tickets):
    """A one-frame strip launch (fewer blocks than CUs: narrow strips, all
    resident at once on an idle GPU) by ticket -- the default for every launch
    size since round 4 -- and by blockIdx, twice in a row; bit-exact."""
    from mvstereovision3_amd import _lib
    rng = np.random.default_rng(9350)
    H, W, D = 200, 520, 128
    L, R = rand_pair(rng, H, W, 30, 0)
    kw = dict(minDisparity=1, numDisparities=D, blockSize=13, P1=2, P2=5, disp12MaxDiff=1,
              uniquenessRatio=0, speckleWindowSize=0, speckleRange=2, mode=1)
    gots = []
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 1)
        _lib.set_option(_lib.OPT_STRIP_TICKETS, tickets)
        for _ in range(2):
            got, want = sgbm_both(mvsv, oracle, L, R, **kw)
            gots.append(got)
    finally:
        _lib.set_option(_lib.OPT_STRIP_TICKETS, 1)
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    for got in gots:
        assert np.array_equal(got, want), f"tickets={tickets}: " + report(got, want)
