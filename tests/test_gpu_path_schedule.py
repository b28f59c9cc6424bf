"""SGBM path schedules of the 16-lane kernels: all line directions side by side
(sgbm_pathdirs16_kernel, one plane per direction: 4-bit when P2 <= 15 --
chosen for launches too small to fill the GPU with sheared strips -- bytes or
u16 when forced with larger P2) against the sheared-strip
schedule, both forced on the same inputs and bit-exact against the oracle:
D = 32 / 64 / 128 / 256, 5 and 8 paths, the no-wrap and the general
recurrence, uniqueness, a frame batch through the device path.
Reference: Disparity::sgbm (src/disparity.cpp:6-10) -> cv::StereoSGBM::compute."""
import numpy as np
import pytest

from tests.test_gpu_parity import rand_pair, report, sgbm_both

pytestmark = pytest.mark.gpu

CASES = [
    # (H, W, D, blockSize, P1, P2, mode)
    (50, 150, 32, 3, 2, 5, 1),
    (61, 200, 64, 5, 0, 0, 0),        # OpenCV defaults P1 = 2, P2 = 5
    (90, 300, 128, 13, 2, 5, 1),      # configs/sgbm.yml shape
    (45, 260, 128, 7, 4, 15, 0),      # largest P2 of the side-by-side schedule
    (40, 420, 256, 9, 2, 5, 1),       # D = 256
    (36, 140, 64, 21, 2, 5, 1),       # general (wrapping) recurrence
    (48, 220, 128, 5, 8, 100, 1),     # forced side by side: byte planes
    (40, 330, 256, 9, 648, 2592, 0),  # forced side by side: u16 planes (config 5 params)
]


@pytest.mark.parametrize("sched", [1, 2])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_path_schedule_forced(gpu, mvsv, oracle, case, sched):
    from mvstereovision3_amd import _lib
    H, W, D, bs, P1, P2, mode = CASES[case]
    rng = np.random.default_rng(9300 + 11 * case)
    L, R = rand_pair(rng, H, W, int(rng.integers(0, min(D, 48))), int(rng.integers(0, 3)))
    kw = dict(minDisparity=int(rng.integers(-3, 3)), numDisparities=D, blockSize=bs, P1=P1, P2=P2,
              disp12MaxDiff=int(rng.integers(-1, 3)), uniquenessRatio=int(rng.choice([0, 10])),
              speckleWindowSize=int(rng.choice([0, 20])), speckleRange=2, mode=mode)
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, sched)
        got, want = sgbm_both(mvsv, oracle, L, R, variant=int(rng.integers(0, 4)), **kw)
    finally:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    assert np.array_equal(got, want), f"schedule={sched} {kw}: " + report(got, want)


def test_path_schedule_batch_device(gpu, mvsv, oracle):
    from mvstereovision3_amd import _lib
    torch = gpu
    rng = np.random.default_rng(9400)
    H, W, D = 80, 240, 128
    pairs = [rand_pair(rng, H, W, int(rng.integers(0, 40)), k % 3) for k in range(3)]
    m = mvsv.StereoSGBM.create(minDisparity=1, numDisparities=D, blockSize=13, P1=2, P2=5,
                               disp12MaxDiff=1, uniquenessRatio=5, mode=1)
    dev = torch.device("cuda", 0)
    Lb = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
    Rb = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
    out = torch.empty((3, H, W), dtype=torch.int16, device=dev)
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 2)
        m.compute(Lb, Rb, out)
        got = out.cpu().numpy()
    finally:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    p = dict(min_disparity=1, num_disparities=D, block_size=13, p1=2, p2=5, disp12_max_diff=1,
             pre_filter_cap=0, uniqueness_ratio=5, speckle_window_size=0, speckle_range=0, mode=1)
    for i, (L, R) in enumerate(pairs):
        want = oracle.sgbm(L, R, p)
        assert np.array_equal(got[i], want), f"frame {i}: " + report(got[i], want)


def test_path_schedule_option_range(gpu):
    from mvstereovision3_amd import _lib
    for bad in (-1, 3):
        with pytest.raises(_lib.MvsvError):
            _lib.set_option(_lib.OPT_PATH_SCHEDULE, bad)
    for bad in (-1, 65):
        with pytest.raises(_lib.MvsvError):
            _lib.set_option(_lib.OPT_STRIP_WAVES, bad)
    with pytest.raises(_lib.MvsvError):
        _lib.set_option(99, 0)  # unknown option
