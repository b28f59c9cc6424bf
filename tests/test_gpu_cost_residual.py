"""Cost residual plane (round 4): the SGBM direction passes read
R = min(C - min_d C, 2*P2) + P2 in nibbles instead of the int16 cost volume C
wherever that is exact (no-wrap regime, 3*P2 <= 15, numDisparities <= 128 --
configs/sgbm.yml).  Every case runs with the residual on (the default) and
forced off (MVSV_OPT_COST_RESIDUAL = 0), under both 16-lane path schedules
(sheared strips + L->R lines, directions side by side), and both must be
bit-exact against the oracle: the plane changes bytes, never results.
Reference: Disparity::sgbm (src/disparity.cpp:6-10) -> cv::StereoSGBM::compute;
mode from loadSGBMParameters (src/disparity.cpp:92-95)."""
import numpy as np
import pytest

from tests.test_gpu_parity import rand_pair, report, sgbm_both

pytestmark = pytest.mark.gpu

CASES = [
    # (H, W, D, blockSize, P1, P2, mode, minD)
    (50, 150, 32, 3, 2, 5, 1, 0),
    (61, 200, 64, 5, 0, 0, 0, 1),       # OpenCV defaults P1 = 2, P2 = 5 (MODE_SGBM fix-ups)
    (90, 300, 128, 13, 2, 5, 1, 1),     # configs/sgbm.yml shape, MODE_HH
    (77, 290, 128, 13, 0, 0, 0, 1),     # configs/sgbm.yml as loaded (mode 0)
    (40, 260, 128, 9, 1, 3, 1, -2),     # small P2, negative minDisparity
    (33, 180, 64, 15, 2, 5, 0, 0),      # largest register-ring window
    (45, 220, 128, 7, 2, 6, 1, 0),      # 3*P2 > 15: residual not used (same results)
]


@pytest.mark.parametrize("res", [1, 0])
@pytest.mark.parametrize("sched", [1, 2])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_cost_residual_forced(gpu, mvsv, oracle, case, sched, res):
    from mvstereovision3_amd import _lib
    H, W, D, bs, P1, P2, mode, minD = CASES[case]
    rng = np.random.default_rng(9700 + 13 * case)
    kind = case % 3  # textured, low texture (ties / flat costs), third generator
    L, R = rand_pair(rng, H, W, int(rng.integers(0, min(D, 40))), kind)
    kw = dict(minDisparity=minD, numDisparities=D, blockSize=bs, P1=P1, P2=P2,
              disp12MaxDiff=int(rng.integers(-1, 3)), uniquenessRatio=int(rng.choice([0, 10])),
              speckleWindowSize=int(rng.choice([0, 20])), speckleRange=2, mode=mode)
    variant = int(rng.integers(0, 4))
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, sched)
        _lib.set_option(_lib.OPT_COST_RESIDUAL, res)
        got, want = sgbm_both(mvsv, oracle, L, R, variant=variant, **kw)
    finally:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
        _lib.set_option(_lib.OPT_COST_RESIDUAL, 1)
    assert np.array_equal(got, want), f"residual={res} schedule={sched} variant={variant} {kw}: " + report(got, want)


def test_cost_residual_batch_device(gpu, mvsv, oracle):
    """A 3-frame batch on the device path with strips (the bench's schedule)."""
    from mvstereovision3_amd import _lib
    torch = gpu
    rng = np.random.default_rng(9800)
    H, W, D = 96, 320, 128
    pairs = [rand_pair(rng, H, W, int(rng.integers(0, 40)), k % 3) for k in range(3)]
    m = mvsv.StereoSGBM.create(minDisparity=1, numDisparities=D, blockSize=13, P1=2, P2=5,
                               disp12MaxDiff=1, uniquenessRatio=0, mode=1)
    dev = torch.device("cuda", 0)
    Lb = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
    Rb = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
    outs = []
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 1)
        for res in (1, 0):
            _lib.set_option(_lib.OPT_COST_RESIDUAL, res)
            out = torch.empty((3, H, W), dtype=torch.int16, device=dev)
            m.compute(Lb, Rb, out)
            outs.append(out.cpu().numpy())
    finally:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
        _lib.set_option(_lib.OPT_COST_RESIDUAL, 1)
    p = dict(min_disparity=1, num_disparities=D, block_size=13, p1=2, p2=5, disp12_max_diff=1,
             pre_filter_cap=0, uniqueness_ratio=0, speckle_window_size=0, speckle_range=0, mode=1)
    assert np.array_equal(outs[0], outs[1])
    for i, (L, R) in enumerate(pairs):
        want = oracle.sgbm(L, R, p)
        assert np.array_equal(outs[0][i], want), f"frame {i}: " + report(outs[0][i], want)


def test_cost_residual_option_range(gpu):
    from mvstereovision3_amd import _lib
    for bad in (-1, 2):
        with pytest.raises(_lib.MvsvError):
            _lib.set_option(_lib.OPT_COST_RESIDUAL, bad)
