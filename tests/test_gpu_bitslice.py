"""Bit-sliced path aggregation (round 5 MODE_HH, round 6 MODE_SGBM; mvsv_bsgm.hip):
where it applies (MODE_HH or MODE_SGBM, numDisparities 128, P1 2 / P2 5 -- configs/sgbm.yml's effective penalties
--, uniquenessRatio 0, no int16 wrap) the six strip directions, the two row
directions and the WTA run on bit planes.  Every case runs with the bit-sliced
path on strips (frame batches), side by side (small launches) and forced off
(MVSV_OPT_BITSLICE = 0, the packed int16 kernels), and all must be bit-exact
against the oracle.
Reference: Disparity::sgbm (src/disparity.cpp:6-10) -> cv::StereoSGBM::compute;
mode from loadSGBMParameters (src/disparity.cpp:92-95)."""
import numpy as np
import pytest

from tests.test_gpu_parity import rand_pair, report, sgbm_both

pytestmark = pytest.mark.gpu

CASES = [
    # (H, W, blockSize, P1, P2, minD, disp12)
    (40, 200, 13, 2, 5, 1, 0),      # configs/sgbm.yml shape (P1 / P2 given)
    (53, 231, 13, 0, 0, 1, 0),      # sgbm.yml as loaded: P1 = P2 = 0 -> 2 / 5
    (31, 190, 3, 2, 5, 0, 2),       # small window
    (64, 300, 15, 0, 0, -3, 1),     # largest register-ring window, negative minDisparity
    (17, 140, 9, 2, 5, 4, -1),      # short image: few strips, chain of one
    (120, 420, 11, 0, 0, 1, 3),     # several strips per chain, both passes
    (9, 135, 5, 0, 0, 0, 0),        # fewer rows than the window (pinned rows only)
    (90, 129 + 127, 7, 2, 5, 0, 0), # W1 = 128: a single strip column group edge
]


# (bit-sliced, path schedule): strips (1), side by side (2: each direction on its
# own chains, the small-launch form), the packed int16 kernels on strips
@pytest.mark.parametrize("bits,sched", [(1, 1), (1, 2), (0, 1)])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_bitslice_hh_forced(gpu, mvsv, oracle, case, bits, sched):
    from mvstereovision3_amd import _lib
    H, W, bs, P1, P2, minD, d12 = CASES[case]
    rng = np.random.default_rng(5100 + 7 * case)
    kind = case % 3
    L, R = rand_pair(rng, H, W, int(rng.integers(0, 60)), kind)
    kw = dict(minDisparity=minD, numDisparities=128, blockSize=bs, P1=P1, P2=P2, disp12MaxDiff=d12,
              uniquenessRatio=0, speckleWindowSize=int(rng.choice([0, 20])), speckleRange=2, mode=1)
    variant = int(rng.integers(0, 4))
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, sched)
        _lib.set_option(_lib.OPT_BITSLICE, bits)
        got, want = sgbm_both(mvsv, oracle, L, R, variant=variant, **kw)
    finally:
        _lib.set_option(_lib.OPT_BITSLICE, 1)
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    assert np.array_equal(got, want), f"bitslice={bits} sched={sched} variant={variant} {kw}: " + report(got, want)


@pytest.mark.parametrize("groups", ["1", "2", "3", "4", "5", "2-serial", "2-nofuse", "2-mode0", "3-mode0", "1-mode0-nofuse"])
def test_bitslice_strip_groups(gpu, mvsv, oracle, groups, monkeypatch):
    """Every strip width (column groups per strip) on a 3-frame device batch;
    -serial: the L->R lines after the strips on the context stream instead of
    beside them; -nofuse: both line directions in the line kernel and the
    separate WTA instead of R->L fused with the WTA."""
    from mvstereovision3_amd import _lib
    torch = gpu
    monkeypatch.setenv("MVSV_BS_GROUPS", groups.split("-")[0])
    monkeypatch.setenv("MVSV_BS_SERIAL", "1" if groups.endswith("serial") else "0")
    monkeypatch.setenv("MVSV_BS_FUSE", "0" if groups.endswith("nofuse") else "1")
    monkeypatch.setenv("MVSV_PATH_SCHEDULE", "1")
    ctx = _lib.Context(0)  # a fresh context reads the environment
    rng = np.random.default_rng(5200 + len(groups) + int(groups[0]))
    H, W, D = 72, 330, 128
    pairs = [rand_pair(rng, H, W, int(rng.integers(0, 50)), k % 3) for k in range(3)]
    mode = 0 if "mode0" in groups else 1
    m = mvsv.StereoSGBM.create(minDisparity=1, numDisparities=D, blockSize=13, P1=0, P2=0, disp12MaxDiff=0,
                               uniquenessRatio=0, mode=mode)
    dev = torch.device("cuda", 0)
    Lb = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
    Rb = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
    out = torch.empty((3, H, W), dtype=torch.int16, device=dev)
    try:
        with _lib.use_context(ctx):
            m.compute(Lb, Rb, out)
            _lib.synchronize(0)
        got = out.cpu().numpy()
    finally:
        ctx.close()
    p = dict(min_disparity=1, num_disparities=D, block_size=13, p1=0, p2=0, disp12_max_diff=0,
             pre_filter_cap=0, uniqueness_ratio=0, speckle_window_size=0, speckle_range=0, mode=mode)
    for i, (L, R) in enumerate(pairs):
        want = oracle.sgbm(L, R, p)
        assert np.array_equal(got[i], want), f"groups={groups} frame {i}: " + report(got[i], want)


# MODE_SGBM (5 paths: the down pass's three directions and both row directions),
# the mode configs/sgbm.yml selects (mode 0 -> src/disparity.cpp:92-95), under
# each OpenCV variant: 0 = 3.4 (lane tie rule d mod 8, column 0 and the bottom
# rows copied), 1 = FIRSTCOL_FIX, 2 = WTA_MIN_D (smallest d on ties)
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("bits,sched", [(1, 1), (1, 2), (0, 1)])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_bitslice_sgbm5_forced(gpu, mvsv, oracle, case, bits, sched, variant):
    from mvstereovision3_amd import _lib
    H, W, bs, P1, P2, minD, d12 = CASES[case]
    rng = np.random.default_rng(6100 + 7 * case + variant)
    kind = (case + variant) % 3
    L, R = rand_pair(rng, H, W, int(rng.integers(0, 60)), kind)
    kw = dict(minDisparity=minD, numDisparities=128, blockSize=bs, P1=P1, P2=P2, disp12MaxDiff=d12,
              uniquenessRatio=0, speckleWindowSize=int(rng.choice([0, 20])), speckleRange=2, mode=0)
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, sched)
        _lib.set_option(_lib.OPT_BITSLICE, bits)
        got, want = sgbm_both(mvsv, oracle, L, R, variant=variant, **kw)
    finally:
        _lib.set_option(_lib.OPT_BITSLICE, 1)
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    assert np.array_equal(got, want), f"bitslice={bits} sched={sched} variant={variant} {kw}: " + report(got, want)


@pytest.mark.parametrize("mode", [1, 0])
def test_bench_batch_every_frame(gpu, mvsv, oracle, mode):
    """The benchmarked code path pinned frame by frame: BASELINE config 4's per-GPU
    share (8 x 1280x960, D 128, configs/sgbm.yml values, the bench's synthetic
    frames) as ONE device launch on the strip schedule with the bit-sliced
    kernels (mode 1 = the bench workload, mode 0 = what sgbm.yml selects), every
    frame against the oracle (8 oracle threads)."""
    import threading
    from mvstereovision3_amd import _lib
    torch = gpu
    SEED0 = 0x5EED0000
    frames = [mvsv.synth_pair(SEED0 + i, 1280, 960, 1, 128) for i in range(8)]
    dev = torch.device("cuda", 0)
    Lt = torch.from_numpy(np.stack([f[0] for f in frames])).to(dev)
    Rt = torch.from_numpy(np.stack([f[1] for f in frames])).to(dev)
    m = mvsv.StereoSGBM.create(1, 128, 13, 0, 0, 0, 0, 0, 150, 2, mode)
    try:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 1)
        _lib.set_option(_lib.OPT_BITSLICE, 1)
        got = m.compute(Lt, Rt)
        torch.cuda.synchronize()
        got = got.cpu().numpy()
    finally:
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    p = dict(m.params())
    p.pop("variant")
    want = [None] * 8

    def run(i):
        want[i] = oracle.sgbm(frames[i][0], frames[i][1], p)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for i in range(8):
        assert np.array_equal(got[i], want[i]), f"mode {mode} frame {i}: " + report(got[i], want[i])


def test_bitslice_option_range(gpu):
    from mvstereovision3_amd import _lib
    for bad in (-1, 2):
        with pytest.raises(_lib.MvsvError):
            _lib.set_option(_lib.OPT_BITSLICE, bad)


@pytest.mark.parametrize("shape", [(1, 480, 640), (8, 240, 640)])
def test_bitslice_workspace_bound(gpu, mvsv, shape):
    """mvsv_sgbm_workspace_bytes bounds what a fresh context allocates for one
    bit-sliced call (side by side for the single frame, strips for the batch)."""
    import ctypes
    from mvstereovision3_amd import _lib
    torch = gpu
    n, H, W = shape
    m = mvsv.StereoSGBM.create(minDisparity=1, numDisparities=128, blockSize=13, P1=0, P2=0,
                               uniquenessRatio=0, speckleWindowSize=150, speckleRange=2, mode=1)
    est = _lib.lib().mvsv_sgbm_workspace_bytes(n, W, H, ctypes.byref(m._params))
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5300 + n)
    L = torch.from_numpy(rng.integers(0, 256, (n, H, W), dtype=np.uint8)).to(dev)
    R = torch.roll(L, -20, dims=2).contiguous()
    out = torch.empty((n, H, W), dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    ctx = _lib.Context(0)
    try:
        free0 = torch.cuda.mem_get_info()[0]
        with _lib.use_context(ctx):
            m.compute(L, R, out)
            _lib.synchronize(0)
        used = free0 - torch.cuda.mem_get_info()[0]
    finally:
        ctx.close()
    # allocation granularity / runtime slack: 64 MB
    assert used <= est + (64 << 20), f"context used {used} B, workspace estimate {est} B"


def test_sgbm_plan_reports_the_pipeline(gpu, mvsv):
    """mvsv_sgbm_plan (what bench.py's byte model reads): the bit-sliced strips
    for the headline batch, the bit-sliced side-by-side chains for one camera
    frame and for the 5-path 640x480 batch, the packed strips with the residual
    plane when bit-slicing is off, and no bit-slicing for config 5."""
    from mvstereovision3_amd import _lib
    ctx = _lib.context(0)
    hh = mvsv.StereoSGBM.create(1, 128, 13, 0, 0, 0, 0, 0, 150, 2, 1)
    sg = mvsv.StereoSGBM.create(1, 128, 13, 0, 0, 0, 0, 0, 150, 2, 0)
    c5 = mvsv.StereoSGBM.create(0, 256, 9, 648, 2592)
    B, SIDE, STRIPS, RES = _lib.PLAN_BITSLICE, _lib.PLAN_SIDE, _lib.PLAN_STRIPS, _lib.PLAN_RESIDUAL
    assert _lib.sgbm_plan(ctx, 8, 1280, 960, hh._params) == B | STRIPS
    assert _lib.sgbm_plan(ctx, 8, 1280, 960, sg._params) == B | STRIPS
    assert _lib.sgbm_plan(ctx, 1, 640, 480, hh._params) == B | SIDE
    assert _lib.sgbm_plan(ctx, 8, 640, 480, sg._params) == B | SIDE
    assert _lib.sgbm_plan(ctx, 8, 1280, 960, c5._params) & B == 0
    try:
        _lib.set_option(_lib.OPT_BITSLICE, 0)
        assert _lib.sgbm_plan(ctx, 8, 1280, 960, hh._params) == STRIPS | RES
    finally:
        _lib.set_option(_lib.OPT_BITSLICE, 1)
