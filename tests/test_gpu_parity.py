"""HIP path vs the CPU oracle, bit-exact (int16 disparity x 16).

Every test calls the kernels through the C ABI (libmvsv.so via the host mirror
in mvstereovision3_amd.disparity) and compares with oracle/ (OpenCV 3.4
restatement; parity unpinned, see oracle/mvsv_oracle.h).  Sizes: random small
cases in the seconds range for the oracle, plus the BASELINE.json configs at
full size (640x480 and 1280x960).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED0 = 0x5EED0000


def report(a, b):
    bad = np.argwhere(a != b)
    if bad.size == 0:
        return ""
    pts = [(int(y), int(x), int(a[y, x]), int(b[y, x])) for y, x in bad[:10]]
    return f"{len(bad)} mismatches of {a.size}; first (y, x, gpu, oracle): {pts}"


def sgbm_both(mvsv, oracle, L, R, variant=0, **kw):
    names = dict(minDisparity="min_disparity", numDisparities="num_disparities",
                 blockSize="block_size", P1="p1", P2="p2", disp12MaxDiff="disp12_max_diff",
                 preFilterCap="pre_filter_cap", uniquenessRatio="uniqueness_ratio",
                 speckleWindowSize="speckle_window_size", speckleRange="speckle_range", mode="mode")
    m = mvsv.StereoSGBM.create(**kw)
    m.setVariant(variant)
    got = m.compute(L, R)
    p = {v: int(kw.get(k, d)) for (k, v), d in zip(names.items(),
                                                    (0, 16, 3, 0, 0, 0, 0, 0, 0, 0, 0))}
    want = oracle.sgbm(L, R, p, flags=variant)
    return got, want


def bm_both(mvsv, oracle, L, R, p):
    m = mvsv.StereoBM.create(p["num_disparities"], p["block_size"])
    m._params.pre_filter_type = p["pre_filter_type"]
    m._params.pre_filter_size = p["pre_filter_size"]
    m._params.pre_filter_cap = p["pre_filter_cap"]
    m._params.min_disparity = p["min_disparity"]
    m._params.texture_threshold = p["texture_threshold"]
    m._params.uniqueness_ratio = p["uniqueness_ratio"]
    m._params.speckle_window_size = p["speckle_window_size"]
    m._params.speckle_range = p["speckle_range"]
    m._params.disp12_max_diff = p["disp12_max_diff"]
    return m.compute(L, R), oracle.bm(L, R, p)


def rand_pair(rng, H, W, shift, kind):
    if kind == 0:
        from scipy.ndimage import uniform_filter
        L = uniform_filter(rng.integers(0, 256, (H, W)).astype(float), 3).round().astype(np.uint8)
    elif kind == 1:  # low texture: ties, texture filter, saturation
        L = (rng.integers(0, 4, (H, W)) * 60).astype(np.uint8)
        L[:, W // 3:W // 2] = 128
    else:
        L = rng.integers(0, 256, (H, W)).astype(np.uint8)
    R = np.roll(L, -shift, axis=1)
    R = np.clip(R.astype(int) + rng.integers(-2, 3, R.shape), 0, 255).astype(np.uint8)
    return L, R


# ---------------------------------------------------------------- SGBM -----
@pytest.mark.parametrize("seed", range(24))
def test_sgbm_random_small(gpu, mvsv, oracle, seed):
    rng = np.random.default_rng(1000 + seed)
    H, W = int(rng.integers(12, 70)), int(rng.integers(48, 120))
    D = int(rng.choice([16, 32, 48, 64]))
    kw = dict(minDisparity=int(rng.integers(-6, 6)), numDisparities=D,
              blockSize=int(rng.choice([0, 1, 3, 5, 7, 9, 11])),
              P1=int(rng.choice([0, 2, 72, 300])), P2=int(rng.choice([0, 5, 288, 2000, 4000])),
              disp12MaxDiff=int(rng.integers(-1, 4)),
              preFilterCap=int(rng.choice([0, 15, 31, 63])),
              uniquenessRatio=int(rng.choice([-1, 0, 5, 15])),
              speckleWindowSize=int(rng.choice([0, 10, 50])),
              speckleRange=int(rng.choice([1, 2, 4])), mode=int(rng.integers(0, 2)))
    if W + min(kw["minDisparity"], 0) - max(kw["minDisparity"] + D, 0) <= max(kw["blockSize"], 5) // 2:
        kw["numDisparities"] = 16
    L, R = rand_pair(rng, H, W, int(rng.integers(0, 16)), int(rng.integers(0, 3)))
    variant = int(rng.integers(0, 4))
    got, want = sgbm_both(mvsv, oracle, L, R, variant=variant, **kw)
    assert np.array_equal(got, want), f"{kw} variant={variant}: " + report(got, want)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("D", [16, 128, 256])
def test_sgbm_synthetic_modes(gpu, mvsv, oracle, mode, D):
    L, R = mvsv.synth_pair(SEED0 + D, 320, 96, 0, D) if D < 256 else \
        mvsv.synth_pair(SEED0 + D, 400, 64, 0, D)
    got, want = sgbm_both(mvsv, oracle, L, R, minDisparity=0, numDisparities=D, blockSize=9,
                          P1=8 * 81, P2=32 * 81, uniquenessRatio=5, speckleWindowSize=40,
                          speckleRange=2, mode=mode)
    assert np.array_equal(got, want), report(got, want)


@pytest.mark.parametrize("seed", range(8))
def test_sgbm_wide_disparity_odd_rows(gpu, mvsv, oracle, seed):
    # D >= 128 runs the 32-lanes-per-row final kernel (two image rows per wave,
    # buffer-descriptor prefetch): odd heights leave the last wave half-empty
    rng = np.random.default_rng(7000 + seed)
    D = 128 if seed < 6 else 256
    H = int(rng.integers(9, 60)) | 1
    W = D + int(rng.integers(40, 90))
    kw = dict(minDisparity=int(rng.integers(-4, 4)), numDisparities=D,
              blockSize=int(rng.choice([1, 3, 5, 9, 13])),
              P1=int(rng.choice([0, 8, 72])), P2=int(rng.choice([0, 5, 288, 2000])),
              disp12MaxDiff=int(rng.integers(-1, 3)), preFilterCap=int(rng.choice([0, 31, 63])),
              uniquenessRatio=int(rng.choice([0, 5, 15])),
              speckleWindowSize=int(rng.choice([0, 20])), speckleRange=2, mode=int(rng.integers(0, 2)))
    L, R = rand_pair(rng, H, W, int(rng.integers(0, 24)), int(rng.integers(0, 3)))
    got, want = sgbm_both(mvsv, oracle, L, R, **kw)
    assert np.array_equal(got, want), f"{kw} H={H} W={W}: " + report(got, want)


@pytest.mark.parametrize("bs", [13, 15, 17, 21])
@pytest.mark.parametrize("D", [64, 128])
def test_sgbm_block_sizes(gpu, mvsv, oracle, bs, D):
    # blockSize <= 15: register-ring cost kernel; larger: the LDS-ring kernel
    L, R = mvsv.synth_pair(SEED0 + bs, 360, 80, 0, D)
    got, want = sgbm_both(mvsv, oracle, L, R, minDisparity=1, numDisparities=D, blockSize=bs,
                          uniquenessRatio=10, speckleWindowSize=30, speckleRange=2, mode=bs & 1 ^ 1)
    assert np.array_equal(got, want), report(got, want)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("D,P2", [(32, 0), (64, 5), (128, 0), (256, 5), (64, 6), (128, 3)])
def test_sgbm_accumulator_plane_formats(gpu, mvsv, oracle, mode, D, P2):
    """Sheared-strip schedule: 4-bit planes when 3 * P2 <= 15 (P2 = 0 -> OpenCV's 5,
    sgbm.yml's case), u8 planes above (P2 = 6), for every D the strip kernels cover."""
    W = 420 if D == 256 else 300
    L, R = mvsv.synth_pair(SEED0 + 13 * D + P2, W, 72, 0, D)
    got, want = sgbm_both(mvsv, oracle, L, R, minDisparity=2, numDisparities=D, blockSize=7,
                          P1=2 if P2 == 3 else 0, P2=P2, uniquenessRatio=10, speckleWindowSize=20,
                          speckleRange=2, mode=mode)
    assert np.array_equal(got, want), report(got, want)


@pytest.mark.parametrize("D", [16, 512])
def test_sgbm_staging_two_slots(gpu, mvsv, oracle, D):
    # shapes whose cost-kernel staging needs two items per thread
    W = 700 if D == 512 else 600
    L, R = mvsv.synth_pair(SEED0 + 7 * D, W, 40, 0, D)
    got, want = sgbm_both(mvsv, oracle, L, R, minDisparity=-3, numDisparities=D, blockSize=7,
                          P1=200, P2=800, mode=1)
    assert np.array_equal(got, want), report(got, want)


def test_sgbm_all_invalid_when_no_columns(gpu, mvsv, oracle):
    L, R = mvsv.synth_pair(SEED0, 40, 20, 0, 64)
    got, want = sgbm_both(mvsv, oracle, L, R, minDisparity=0, numDisparities=64, blockSize=5)
    assert np.array_equal(got, want)
    assert (got == -16).all()


def test_sgbm_roi_views(gpu, mvsv, oracle):
    """Stereopair images are cropped cv::Mat views (stride != width)."""
    big_L, big_R = mvsv.synth_pair(SEED0 + 7, 300, 120, 0, 64)
    L, R = big_L[10:100, 20:260], big_R[10:100, 20:260]
    assert L.strides[0] == 300
    got, want = sgbm_both(mvsv, oracle, L, R, minDisparity=0, numDisparities=64, blockSize=7)
    assert np.array_equal(got, want), report(got, want)


def test_sgbm_reference_call_sites(gpu, mvsv, oracle):
    """liveDisparity create(0,64,9,8*81,32*81) and captureDisparity create(0,16,5,200,800)."""
    L, R = mvsv.synth_pair(SEED0 + 3, 376, 240, 0, 64)  # 2x2-binned mvBlueFOX size
    for kw in (dict(minDisparity=0, numDisparities=64, blockSize=9, P1=648, P2=2592),
               dict(minDisparity=0, numDisparities=16, blockSize=5, P1=200, P2=800)):
        got, want = sgbm_both(mvsv, oracle, L, R, **kw)
        assert np.array_equal(got, want), f"{kw}: " + report(got, want)


def test_sgbm_loader_config(gpu, mvsv, oracle):
    """configs/sgbm.yml through Disparity::loadSGBMParameters + Disparity::sgbm."""
    import os
    from tests.conftest import CONFIGS
    m = mvsv.StereoSGBM.create(0, 0, 0, 8 * 0 * 0, 32 * 0 * 0)  # trgt/mean_test.cpp:233-237
    para = mvsv.sgbmParameters()
    assert mvsv.Disparity.loadSGBMParameters(os.path.join(CONFIGS, "sgbm.yml"), m, para)
    L, R = mvsv.synth_pair(SEED0 + 11, 320, 120, 1, 128)
    out = mvsv.Disparity.sgbm(mvsv.Stereopair(L, R), None, m)
    p = dict(m.params())
    p.pop("variant")
    want = oracle.sgbm(L, R, p)
    assert np.array_equal(out, want), report(out, want)


@pytest.mark.slow
@pytest.mark.parametrize("mode", [0, 1])
def test_sgbm_config3_640x480(gpu, mvsv, oracle, mode):
    """BASELINE config 3: configs/sgbm.yml, 640x480, 128 disparities (mode 0 and 8-path)."""
    L, R = mvsv.synth_pair(SEED0, 640, 480, 1, 128)
    got, want = sgbm_both(mvsv, oracle, L, R, minDisparity=1, numDisparities=128, blockSize=13,
                          disp12MaxDiff=0, preFilterCap=0, uniquenessRatio=0,
                          speckleWindowSize=150, speckleRange=2, mode=mode)
    assert np.array_equal(got, want), report(got, want)


@pytest.mark.slow
def test_sgbm_config4_1280x960_hh(gpu, mvsv, oracle):
    """Headline workload frame: 1280x960, D=128, 8 paths (sgbm.yml values, mode 1)."""
    L, R = mvsv.synth_pair(SEED0 + 1, 1280, 960, 1, 128)
    got, want = sgbm_both(mvsv, oracle, L, R, minDisparity=1, numDisparities=128, blockSize=13,
                          speckleWindowSize=150, speckleRange=2, mode=1)
    assert np.array_equal(got, want), report(got, want)


def test_sgbm_device_batch(gpu, mvsv, oracle):
    """Frame batch on HBM-resident torch tensors == per-frame oracle."""
    torch = gpu
    frames = [mvsv.synth_pair(SEED0 + i, 256, 128, 0, 64) for i in range(3)]
    Lt = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
    Rt = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
    m = mvsv.StereoSGBM.create(0, 64, 7, 8 * 49, 32 * 49, 1, 31, 10, 30, 2, mvsv.MODE_HH)
    out = m.compute(Lt, Rt)
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    p = dict(m.params())
    p.pop("variant")
    for i, (L, R) in enumerate(frames):
        want = oracle.sgbm(L, R, p)
        assert np.array_equal(out[i], want), f"frame {i}: " + report(out[i], want)


# ------------------------------------------------------------------ BM -----
@pytest.mark.parametrize("seed", range(16))
def test_bm_random_small(gpu, mvsv, oracle, seed):
    rng = np.random.default_rng(2000 + seed)
    H, W = int(rng.integers(24, 80)), int(rng.integers(60, 140))
    bs = int(rng.choice([5, 7, 9, 11, 21]))
    if bs >= min(H, W):
        bs = 5
    p = dict(pre_filter_type=1, pre_filter_size=9, pre_filter_cap=int(rng.integers(1, 64)),
             block_size=bs, min_disparity=int(rng.integers(-4, 4)),
             num_disparities=int(rng.choice([16, 32])),
             texture_threshold=int(rng.choice([0, 10, 100])),
             uniqueness_ratio=int(rng.choice([0, 10, 15])),
             speckle_window_size=int(rng.choice([0, 10])),
             speckle_range=int(rng.choice([0, 4, 32])),
             disp12_max_diff=int(rng.choice([-1, 0, 1, 3])))
    L, R = rand_pair(rng, H, W, int(rng.integers(0, 16)), int(rng.integers(0, 3)))
    got, want = bm_both(mvsv, oracle, L, R, p)
    assert np.array_equal(got, want), f"{p}: " + report(got, want)


def bm_defaults(D, bs):
    return dict(pre_filter_type=1, pre_filter_size=9, pre_filter_cap=31, block_size=bs,
                min_disparity=0, num_disparities=D, texture_threshold=10, uniqueness_ratio=15,
                speckle_window_size=0, speckle_range=0, disp12_max_diff=-1)


def test_bm_config1_bm_yml(gpu, mvsv, oracle):
    """BASELINE config 1: configs/bm.yml on a 640x480 pair."""
    import os
    from tests.conftest import CONFIGS
    m = mvsv.StereoBM.create(16, 9)
    assert mvsv.Disparity.loadBMParameters(os.path.join(CONFIGS, "bm.yml"), m)
    L, R = mvsv.synth_pair(SEED0 + 21, 640, 480, 0, 80)
    got = mvsv.Disparity.bm(mvsv.Stereopair(L, R), None, m)
    want = oracle.bm(L, R, m.params())
    assert np.array_equal(got, want), report(got, want)


def test_bm_config2_640x480(gpu, mvsv, oracle):
    """BASELINE config 2: StereoBM::create(64, 9) defaults, 640x480."""
    L, R = mvsv.synth_pair(SEED0 + 22, 640, 480, 0, 64)
    got, want = bm_both(mvsv, oracle, L, R, bm_defaults(64, 9))
    assert np.array_equal(got, want), report(got, want)


@pytest.mark.parametrize("seed", range(8))
def test_bm_normalized_response_prefilter(gpu, mvsv, oracle, seed):
    """StereoBM::PREFILTER_NORMALIZED_RESPONSE (prefilterNorm) on the GPU vs the oracle."""
    rng = np.random.default_rng(3000 + seed)
    H, W = int(rng.integers(40, 120)), int(rng.integers(80, 200))
    p = bm_defaults(int(rng.choice([16, 32])), int(rng.choice([5, 9, 15])))
    p.update(pre_filter_type=0, pre_filter_size=int(rng.choice([5, 7, 9, 21, 31])),
             pre_filter_cap=int(rng.integers(1, 64)), min_disparity=int(rng.integers(-3, 3)),
             texture_threshold=int(rng.choice([0, 10])), disp12_max_diff=int(rng.choice([-1, 1])))
    L, R = rand_pair(rng, H, W, int(rng.integers(0, 12)), int(rng.integers(0, 3)))
    got, want = bm_both(mvsv, oracle, L, R, p)
    assert np.array_equal(got, want), f"{p}: " + report(got, want)


def test_bm_validate_and_speckle(gpu, mvsv, oracle):
    L, R = mvsv.synth_pair(SEED0 + 23, 320, 200, 0, 48)
    p = bm_defaults(48, 11)
    p.update(disp12_max_diff=1, speckle_window_size=60, speckle_range=16, uniqueness_ratio=5)
    got, want = bm_both(mvsv, oracle, L, R, p)
    assert np.array_equal(got, want), report(got, want)


# ---------------------------------------------------------- post-pass ------
def test_mean_disparity_grid(gpu, mvsv, oracle):
    torch = gpu
    L, R = mvsv.synth_pair(SEED0 + 5, 640, 240, 0, 64)
    d = mvsv.StereoSGBM.create(0, 64, 9, 648, 2592).compute(L, R)
    work = d[:, 32:]  # createDMapROIS: x in [numDisp/2, cols)
    got = mvsv.mean_disparity_grid(torch.from_numpy(np.ascontiguousarray(work)).cuda()).cpu().numpy()
    want = oracle.mean_disparity_grid(work)
    assert np.array_equal(got, want)


def test_invalid_params_raise(gpu, mvsv):
    L, R = mvsv.synth_pair(SEED0, 64, 48, 0, 16)
    with pytest.raises(mvsv.MvsvError):
        mvsv.StereoSGBM.create(0, 24, 5).compute(L, R)  # numDisparities % 16 != 0
    with pytest.raises(mvsv.MvsvError):
        mvsv.StereoBM.create(16, 4).compute(L, R)  # even block size


# ------------------------------------------------------ golden fixtures ----
def _fixtures():
    import json
    import os
    from tests.conftest import GOLDEN
    return (np.load(os.path.join(GOLDEN, "fixtures.npz")),
            json.load(open(os.path.join(GOLDEN, "fixtures.json"))))


def test_golden_fixtures_sgbm_bm(gpu, mvsv):
    """Committed vectors (tests/golden/make_golden.py), no oracle in the loop."""
    fix, meta = _fixtures()
    for case in meta["sgbm"]:
        p = case["params"]
        m = mvsv.StereoSGBM.create(p["min_disparity"], p["num_disparities"], p["block_size"],
                                   p["p1"], p["p2"], p["disp12_max_diff"], p["pre_filter_cap"],
                                   p["uniqueness_ratio"], p["speckle_window_size"],
                                   p["speckle_range"], p["mode"])
        m.setVariant(case["variant"])
        got = m.compute(fix[case["name"] + "_L"], fix[case["name"] + "_R"])
        want = fix[case["name"] + "_out"]
        assert np.array_equal(got, want), case["name"] + ": " + report(got, want)
    for case in meta["bm"]:
        p = case["params"]
        m = mvsv.StereoBM.create(p["num_disparities"], p["block_size"])
        for k, v in p.items():
            setattr(m._params, k, v)
        got = m.compute(fix[case["name"] + "_L"], fix[case["name"] + "_R"])
        want = fix[case["name"] + "_out"]
        assert np.array_equal(got, want), case["name"] + ": " + report(got, want)


def test_golden_mean_grid(gpu, mvsv):
    torch = gpu
    fix, _ = _fixtures()
    got = mvsv.mean_disparity_grid(torch.from_numpy(fix["post_in"]).cuda()).cpu().numpy()
    assert np.array_equal(got, fix["post_grid"])


@pytest.mark.slow
def test_size_independent_properties_full_batch(gpu, mvsv):
    """Full-size batch (bench workload, 8 x 1280x960, D=128, 8 paths): batch result
    equals per-frame results, is deterministic across runs, and disparities lie in
    the valid range or are INVALID."""
    torch = gpu
    frames = [mvsv.synth_pair(SEED0 + i, 1280, 960, 1, 128) for i in range(8)]
    Lt = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
    Rt = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
    m = mvsv.StereoSGBM.create(1, 128, 13, 0, 0, 0, 0, 0, 150, 2, mvsv.MODE_HH)
    a = m.compute(Lt, Rt).cpu().numpy()
    b = m.compute(Lt, Rt).cpu().numpy()
    assert np.array_equal(a, b)
    single = m.compute(Lt[5], Rt[5]).cpu().numpy()
    assert np.array_equal(a[5], single)
    valid = a != 0  # INVALID = (minD - 1) * 16 = 0
    assert (a[valid] >= 16).all() and (a[valid] <= 128 * 16 + 16).all()
    # the rectangle of the synthetic field sits at round(0.6 * D) = 77
    assert abs(np.median(a[:, 400:560, 500:800]) / 16 - 77) < 1


# -------------------------------------------------- after the path (f3/f4) -----
def test_reproject_matches_oracle(gpu, mvsv, oracle):
    import json
    import os
    import torch
    from conftest import GOLDEN
    from mvstereovision3_amd.utility import reproject
    Q = np.array(json.load(open(os.path.join(GOLDEN, "q_matrix.json")))["Q"], np.float32)
    L, R = mvsv.synth_pair(SEED0 + 5, 400, 120, 0, 64)
    d = mvsv.StereoSGBM.create(0, 64, 5).compute(L, R)
    d[0, :5] = 0  # W = 0 -> infinite Z -> 0
    d[1, :5] = -16
    got = reproject(torch.from_numpy(d).cuda(), Q).cpu().numpy()
    want = oracle.reproject(d, Q)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    batch = torch.from_numpy(np.stack([d, d[::-1].copy()])).cuda()
    gb = reproject(batch, Q).cpu().numpy()
    assert np.array_equal(gb[1].view(np.uint32), oracle.reproject(d[::-1].copy(), Q).view(np.uint32))


def test_dmap2pcl_writes_reference_ply(gpu, mvsv, oracle, tmp_path):
    import json
    import os
    from conftest import GOLDEN
    from test_utility import ply_text
    from mvstereovision3_amd.utility import Utility
    Q = np.array(json.load(open(os.path.join(GOLDEN, "q_matrix.json")))["Q"], np.float32)
    L, R = mvsv.synth_pair(SEED0 + 6, 200, 60, 0, 32)
    d = mvsv.StereoSGBM.create(0, 32, 5).compute(L, R)
    f = tmp_path / "cloud.ply"
    Utility.dmap2pcl(str(f), d, Q)
    pts = oracle.reproject(d, Q).reshape(-1, 4)
    pts = pts[pts[:, 3] > 0]
    assert f.read_text() == ply_text(pts, 1, "Hagen Hiller", "disparity pointcloud", d)


# ------------------------------------------------------- f1: stream + grid -----
def test_mean_grid_host_map(gpu, mvsv, oracle):
    rng = np.random.default_rng(5)
    d = rng.integers(-16, 3000, (123, 377)).astype(np.int16)
    m = mvsv.MeanDisparityDetection()
    m.init(d.shape, np.eye(4, dtype=np.float32).reshape(16), 0.1, 1.5)
    m.build(d, 0, m.MEAN_VALUE)
    assert np.array_equal(np.array(m.getMeanMap(), np.float32), oracle.mean_disparity_grid(d))


def test_disparity_stream_matches_direct_compute(gpu, mvsv, oracle):
    """Camera loop (trgt/mean_test.cpp:61-70, 258-318) as a depth-3 stream with the ROI grid."""
    W, H = 320, 96
    m = mvsv.StereoSGBM.create(0, 64, 9, 8 * 81, 32 * 81)  # liveDisparity-style parameters
    roi_u, _ = mvsv.create_dmap_rois((H, W), 64)
    st = mvsv.DisparityStream(m, W, H, depth=3, grid_roi=roi_u)
    frames = [mvsv.synth_pair(SEED0 + 40 + i, W, H, 0, 64) for i in range(7)]
    got = []
    for i, (L, R) in enumerate(frames):
        if st.pending() == 3:
            got.append(st.pop())
        if i == 5:  # setters between frames apply to frames pushed afterwards
            m.setUniquenessRatio(15)
            st.set_params(m)
        st.push(L, R)
    while st.pending():
        got.append(st.pop())
    st.close()
    assert len(got) == 7
    for i, ((L, R), (d, means)) in enumerate(zip(frames, got)):
        p = dict(m.params())
        p.pop("variant")
        if i < 5:
            p["uniqueness_ratio"] = 0
        want = oracle.sgbm(L, R, p)
        assert np.array_equal(d, want), f"frame {i}: " + report(d, want)
        x0, y0, x1, y1 = roi_u
        assert np.array_equal(means, oracle.mean_disparity_grid(np.ascontiguousarray(want[y0:y1, x0:x1])))


@pytest.mark.parametrize("depth,batch,inflight", [(4, 2, 1), (5, 3, 1), (6, 6, 1), (6, 2, 2),
                                                  (7, 2, 3), (5, 1, 4)])
def test_disparity_stream_batched(gpu, mvsv, oracle, depth, batch, inflight):
    """Frames computed `batch` at a time, `inflight` launches at once on the stream's
    compute lanes: partial groups on pop, a parameter change mid-group, groups cut
    at the slot ring's end -- every frame still matches."""
    W, H, D = 256, 64, 64
    m = mvsv.StereoSGBM.create(0, D, 7, 8 * 49, 32 * 49)
    roi_u, _ = mvsv.create_dmap_rois((H, W), D)
    st = mvsv.DisparityStream(m, W, H, depth=depth, grid_roi=roi_u, batch=batch, inflight=inflight)
    frames = [mvsv.synth_pair(SEED0 + 60 + i, W, H, 0, D) for i in range(11)]
    got, uq_from = [], 7
    for i, (L, R) in enumerate(frames):
        if st.pending() == depth or i in (3, 4):  # pops that force partial groups
            got.append(st.pop())
        if i == uq_from:
            m.setUniquenessRatio(10)
            st.set_params(m)
        if i == 9 and inflight > 1:
            st.set_inflight(inflight - 1)  # lanes dropped with launches in flight
        st.push(L, R)
    while st.pending():
        got.append(st.pop())
    st.close()
    assert len(got) == len(frames)
    for i, ((L, R), (d, means)) in enumerate(zip(frames, got)):
        p = dict(m.params())
        p.pop("variant")
        if i < uq_from:
            p["uniqueness_ratio"] = 0
        want = oracle.sgbm(L, R, p)
        assert np.array_equal(d, want), f"frame {i}: " + report(d, want)
        x0, y0, x1, y1 = roi_u
        assert np.array_equal(means, oracle.mean_disparity_grid(np.ascontiguousarray(want[y0:y1, x0:x1])))


# ----------------------------------------------------------- f2: remap -----
def test_remap_matches_oracle(gpu, mvsv, oracle):
    import torch
    rng = np.random.default_rng(21)
    H, W = 120, 200
    img = rng.integers(0, 256, (H, W)).astype(np.uint8)
    K = np.array([[150.0, 0, 100], [0, 150.0, 60], [0, 0, 1]])
    R = np.array([[0.9998, -0.01, 0.0174], [0.0102, 0.9999, -0.005], [-0.0174, 0.0052, 0.9998]])
    mx, my = mvsv.init_undistort_rectify_map(K, [-0.25, 0.07, 0.001, -0.0015, 0.0], R, K, (W, H))
    mx[0, :4] = [-3.0, 199.5, 200.2, np.float32(1 / 64)]  # border cases + a half-way rounding
    got = mvsv.remap(torch.from_numpy(img).cuda(), torch.from_numpy(mx).cuda(),
                     torch.from_numpy(my).cuda()).cpu().numpy()
    assert np.array_equal(got, oracle.remap_linear(img, mx, my))


def test_rectify_pair_then_sgbm(gpu, mvsv, oracle):
    """Stereosystem::getRectifiedImagepair + Disparity::sgbm on the cropped pair."""
    L, R = mvsv.synth_pair(SEED0 + 60, 240, 100, 0, 32)
    yy, xx = np.mgrid[0:100, 0:240].astype(np.float32)
    maps = (xx + 0.25, yy, xx - 0.25, yy + 0.5)
    roi = (4, 2, 236, 98)
    rl, rr = mvsv.rectify_pair(L, R, maps, roi)
    x0, y0, x1, y1 = roi
    assert np.array_equal(rl, oracle.remap_linear(L, maps[0], maps[1])[y0:y1, x0:x1])
    assert np.array_equal(rr, oracle.remap_linear(R, maps[2], maps[3])[y0:y1, x0:x1])
    d = mvsv.StereoSGBM.create(0, 32, 5).compute(rl, rr)
    p = dict(mvsv.StereoSGBM.create(0, 32, 5).params())
    p.pop("variant")
    assert np.array_equal(d, oracle.sgbm(rl, rr, p))


def test_stereosystem_rectified_pair_then_sgbm(gpu, mvsv, oracle):
    """Stereosystem::initRectification (stereoRectify + initUndistortRectifyMap from the
    reference's baseline_small calibration files, binning) + getRectifiedImagepair on
    the GPU + Disparity::sgbm of the cropped pair, each step against the oracle."""
    import os
    cal = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "calib", "baseline_small")
    s = mvsv.Stereosystem(376, 240, binning=True)
    assert s.loadIntrinsic(os.path.join(cal, "intrinsic.yml"))
    assert s.loadExtrinisic(os.path.join(cal, "extrinsic.yml"))
    assert s.initRectification()
    L, R = mvsv.synth_pair(SEED0 + 70, 376, 240, 0, 64)
    sip = mvsv.Stereopair(L, R)
    assert s.getRectifiedImagepair(sip)
    x0, y0, x1, y1 = s.mDisplayROI
    assert np.array_equal(sip.mLeft, oracle.remap_linear(L, s.mMap1[0], s.mMap2[0])[y0:y1, x0:x1])
    assert np.array_equal(sip.mRight, oracle.remap_linear(R, s.mMap1[1], s.mMap2[1])[y0:y1, x0:x1])
    m = mvsv.StereoSGBM.create(0, 64, 9, 8 * 81, 32 * 81)
    d = m.compute(sip.mLeft, sip.mRight)
    p = dict(m.params())
    p.pop("variant")
    assert np.array_equal(d, oracle.sgbm(np.ascontiguousarray(sip.mLeft), np.ascontiguousarray(sip.mRight), p))


@pytest.mark.parametrize("threads", ["1", "3"])
def test_stream_copy_pool_and_pop_view(gpu, mvsv, oracle, threads, monkeypatch):
    """Frames large enough for the stream's host copy pool (>= 1 MiB maps), strided
    input rows, pops alternating between a copy (mvsv_stream_pop) and a view of the
    pinned slot (mvsv_stream_pop_view): every map equals the synchronous call's, the
    first also the oracle's, and a view popped after the last push stays intact."""
    monkeypatch.setenv("MVSV_STREAM_COPY_THREADS", threads)
    W, H, D = 1024, 528, 64
    m = mvsv.StereoSGBM.create(0, D, 5, 8 * 25, 32 * 25)
    roi_u, _ = mvsv.create_dmap_rois((H, W), D)
    depth = 3
    st = mvsv.DisparityStream(m, W, H, depth=depth, grid_roi=roi_u)
    frames = []
    for i in range(6):
        L, R = mvsv.synth_pair(SEED0 + 90 + i, W, H, 0, D)
        pad = np.zeros((H, W + 40), np.uint8)
        padR = np.zeros((H, W + 24), np.uint8)
        pad[:, 7:7 + W] = L
        padR[:, 3:3 + W] = R
        frames.append((pad[:, 7:7 + W], padR[:, 3:3 + W]))  # row strides > width
    got = []
    for i, (L, R) in enumerate(frames):
        if st.pending() == depth:
            k = len(got)
            d, means = st.pop(copy_map="view" if k % 2 else True)
            got.append((d.copy(), np.array(d, copy=False), means))
        st.push(L, R)
    while st.pending():
        k = len(got)
        d, means = st.pop(copy_map="view" if k % 2 else True)
        got.append((d.copy(), np.array(d, copy=False), means))
    assert len(got) == len(frames)
    for i, ((L, R), (d, live, means)) in enumerate(zip(frames, got)):
        want = m.compute(np.ascontiguousarray(L), np.ascontiguousarray(R))
        assert np.array_equal(d, want), f"frame {i}: " + report(d, want)
        if i == 0:
            p = dict(m.params())
            p.pop("variant")
            assert np.array_equal(d, oracle.sgbm(np.ascontiguousarray(L), np.ascontiguousarray(R), p))
        x0, y0, x1, y1 = roi_u
        assert np.array_equal(means, oracle.mean_disparity_grid(np.ascontiguousarray(want[y0:y1, x0:x1])))
    # views popped after the last push: still the frame's map
    for i in range(len(frames) - depth, len(frames)):
        if i % 2:
            assert np.array_equal(got[i][1], got[i][0])
    st.close()


def test_stream_pop_view_outlives_close(gpu, mvsv):
    """A pop view keeps the stream's pinned slot alive: close() and
    dropping the stream while the view exists defer the destroy; the view still
    reads the frame's map, and the stream refuses push / pop once closed."""
    W, H, D = 320, 96, 32
    m = mvsv.StereoSGBM.create(0, D, 5, 8 * 25, 32 * 25)
    st = mvsv.DisparityStream(m, W, H, depth=2)
    L, R = mvsv.synth_pair(SEED0 + 97, W, H, 0, D)
    st.push(L, R)
    view, _ = st.pop(copy_map="view")
    want = m.compute(L, R)
    st.close()
    assert st.closed
    with pytest.raises(mvsv.MvsvError):
        st.push(L, R)
    del st
    import gc

    gc.collect()
    assert np.array_equal(view, want)
    del view
    gc.collect()
