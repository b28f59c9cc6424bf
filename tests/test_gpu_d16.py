"""D = 16 on the 8-lanes-per-line kernels (round 6): captureDisparity's
create(0, 16, 5, 200, 800) (trgt/captureDisparity.cpp:24-25,196) and every
plane format of the side-by-side directions (nibbles P2 <= 15, bytes, u16),
both modes, uniqueness, odd heights (the final kernel's eight rows per wave
leave the last wave part-empty), batches -- bit-exact against the oracle."""
import numpy as np
import pytest

from test_gpu_parity import SEED0, rand_pair, report, sgbm_both

pytestmark = pytest.mark.gpu


def test_d16_plan_is_side_by_side(gpu, mvsv):
    from mvstereovision3_amd import _lib
    m = mvsv.StereoSGBM.create(0, 16, 5, 200, 800)
    ctx = _lib.context(0)
    for n in (1, 8):
        plan = _lib.sgbm_plan(ctx, n, 640, 480, m._params)
        assert plan & _lib.PLAN_SIDE and not plan & (_lib.PLAN_BITSLICE | _lib.PLAN_STRIPS), plan


@pytest.mark.parametrize("n", [1, 3])
def test_d16_capture_call_site_640x480(gpu, mvsv, oracle, n):
    torch = gpu
    frames = [mvsv.synth_pair(SEED0 + 160 + i, 640, 480, 0, 16) for i in range(n)]
    m = mvsv.StereoSGBM.create(0, 16, 5, 200, 800)
    Lt = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
    Rt = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
    out = m.compute(Lt, Rt).cpu().numpy()
    p = dict(m.params())
    p.pop("variant")
    for i, (L, R) in enumerate(frames):
        want = oracle.sgbm(L, R, p)
        assert np.array_equal(out[i], want), f"frame {i}: " + report(out[i], want)


@pytest.mark.parametrize("seed", range(16))
def test_d16_random(gpu, mvsv, oracle, seed):
    rng = np.random.default_rng(16000 + seed)
    H = int(rng.integers(9, 90)) | (seed & 1)
    W = int(rng.integers(40, 260))
    kw = dict(minDisparity=int(rng.integers(-5, 5)), numDisparities=16,
              blockSize=int(rng.choice([1, 3, 5, 7, 9, 11])),
              P1=int(rng.choice([0, 2, 8, 200])), P2=int(rng.choice([0, 5, 15, 40, 800, 3000])),
              disp12MaxDiff=int(rng.integers(-1, 3)), preFilterCap=int(rng.choice([0, 15, 63])),
              uniquenessRatio=int(rng.choice([0, 5, 15])),
              speckleWindowSize=int(rng.choice([0, 20])), speckleRange=2, mode=int(rng.integers(0, 2)))
    if W + min(kw["minDisparity"], 0) - max(kw["minDisparity"] + 16, 0) <= kw["blockSize"] // 2:
        W += 40
    L, R = rand_pair(rng, H, W, int(rng.integers(0, 14)), int(rng.integers(0, 3)))
    variant = int(rng.integers(0, 4))
    got, want = sgbm_both(mvsv, oracle, L, R, variant=variant, **kw)
    assert np.array_equal(got, want), f"{kw} H={H} W={W} variant={variant}: " + report(got, want)


@pytest.mark.parametrize("mode", [0, 1])
def test_d16_batch_matches_frames(gpu, mvsv, oracle, mode):
    """Eight 320x241 frames in one launch == the oracle per frame (u16 planes, MODE_HH's
    seven planes)."""
    torch = gpu
    frames = [mvsv.synth_pair(SEED0 + 170 + i, 320, 241, 0, 16) for i in range(8)]
    m = mvsv.StereoSGBM.create(0, 16, 5, 200, 800, 1, 0, 10, 20, 2, mode)
    Lt = torch.from_numpy(np.stack([f[0] for f in frames])).cuda()
    Rt = torch.from_numpy(np.stack([f[1] for f in frames])).cuda()
    out = m.compute(Lt, Rt).cpu().numpy()
    p = dict(m.params())
    p.pop("variant")
    for i in (0, 4, 7):
        want = oracle.sgbm(frames[i][0], frames[i][1], p)
        assert np.array_equal(out[i], want), f"frame {i}: " + report(out[i], want)


@pytest.mark.parametrize("site", ["capture", "live"])
def test_call_site_workspace_bound(gpu, mvsv, site):
    """mvsv_sgbm_workspace_bytes bounds what a fresh context allocates for one frame of
    the reference's call sites (directions side by side on u16 planes, R->L included)."""
    import ctypes
    from mvstereovision3_amd import _lib
    torch = gpu
    n, H, W = (1, 480, 640) if site == "capture" else (1, 960, 1280)
    m = mvsv.StereoSGBM.create(0, 16, 5, 200, 800) if site == "capture" else \
        mvsv.StereoSGBM.create(0, 64, 9, 648, 2592)
    est = _lib.lib().mvsv_sgbm_workspace_bytes(n, W, H, ctypes.byref(m._params))
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5400)
    L = torch.from_numpy(rng.integers(0, 256, (n, H, W), dtype=np.uint8)).to(dev)
    R = torch.roll(L, -9, dims=2).contiguous()
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
    assert used <= est + (64 << 20), f"context used {used} B, workspace estimate {est} B"


@pytest.mark.parametrize("split", ["1", "0"])
def test_call_sites_split_wta_both_forms(gpu, mvsv, oracle, split, monkeypatch):
    """The side-by-side schedule on byte / u16 planes with the R->L direction as a chain
    set and the per-pixel WTA kernel (MVSV_FINAL_SPLIT=1, default; D <= 32) and with the
    fused R->L + WTA final kernel (0, and D > 32 either way): bit-exact, both modes,
    uniqueness on and off, byte and u16 planes."""
    from mvstereovision3_amd import _lib
    monkeypatch.setenv("MVSV_FINAL_SPLIT", split)
    ctx = _lib.Context(0)
    try:
        with _lib.use_context(ctx):
            for i, (D, bs, P1, P2, uq, mode, W, H) in enumerate(
                    [(16, 5, 200, 800, 0, 0, 320, 97), (64, 9, 648, 2592, 0, 0, 360, 64),
                     (32, 7, 8, 40, 10, 1, 300, 51), (64, 5, 72, 300, 15, 1, 280, 40),
                     (16, 3, 8, 20, 5, 0, 200, 33), (32, 3, 8, 30, 0, 1, 200, 33),
                     (128, 9, 648, 2592, 10, 0, 420, 40)]):
                L, R = mvsv.synth_pair(SEED0 + 180 + i, W, H, 0, D)
                kw = dict(minDisparity=i - 2, numDisparities=D, blockSize=bs, P1=P1, P2=P2,
                          uniquenessRatio=uq, disp12MaxDiff=1, speckleWindowSize=20, speckleRange=2, mode=mode)
                for variant in (0, 2):
                    got, want = sgbm_both(mvsv, oracle, L, R, variant=variant, **kw)
                    assert np.array_equal(got, want), f"split={split} {kw} variant={variant}: " + report(got, want)
    finally:
        ctx.close()
