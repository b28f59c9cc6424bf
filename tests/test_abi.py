"""C-ABI checks that need no GPU: libmvsv.so loads, exports every symbol that
include/mvsv.h declares, and the host-side entry points (parameter defaults /
validation with OpenCV's rules, the YAML loaders, the synthetic generator)
behave as specified.  No compute is launched here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from tests.conftest import CONFIGS, ROOT


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "mvsv.h")).read()
    return sorted(set(re.findall(r"MVSV_API\s+[\w\s\*]+?\b(mvsv_\w+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol(mvsv):
    from mvstereovision3_amd import _lib
    lib = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mvsv_\w+)", out))
    assert set(syms) <= exported
    assert exported <= set(syms), f"undeclared exports: {exported - set(syms)}"


def test_library_is_gfx950_code_object(mvsv):
    from mvstereovision3_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"--gfx9" not in data.replace(b"--gfx950", b"")  # no other offload targets


def test_version(mvsv):
    from mvstereovision3_amd import _lib
    assert _lib.lib().mvsv_version() == 100


def test_sgbm_create_defaults(mvsv):
    m = mvsv.StereoSGBM.create()
    assert m.params() == dict(min_disparity=0, num_disparities=16, block_size=3, p1=0, p2=0,
                              disp12_max_diff=0, pre_filter_cap=0, uniqueness_ratio=0,
                              speckle_window_size=0, speckle_range=0, mode=0, variant=0)
    live = mvsv.StereoSGBM.create(0, 64, 9, 8 * 81, 32 * 81)  # trgt/liveDisparity.cpp:61
    assert live.getP1() == 648 and live.getP2() == 2592 and live.getBlockSize() == 9


def test_bm_create_defaults(mvsv):
    b = mvsv.StereoBM.create(64, 9)
    assert b.params() == dict(pre_filter_type=1, pre_filter_size=9, pre_filter_cap=31,
                              block_size=9, min_disparity=0, num_disparities=64,
                              texture_threshold=10, uniqueness_ratio=15, speckle_window_size=0,
                              speckle_range=0, disp12_max_diff=-1)
    assert mvsv.StereoBM.create(0, 21).getNumDisparities() == 64


@pytest.mark.parametrize("D,ok", [(16, True), (128, True), (0, False), (24, False), (-16, False)])
def test_sgbm_validation(mvsv, D, ok):
    from mvstereovision3_amd import _lib
    m = mvsv.StereoSGBM.create(0, D, 5)
    rc = _lib.lib().mvsv_sgbm_validate(ctypes.byref(m._params), 640, 480)
    assert (rc == 0) == ok


@pytest.mark.parametrize("field,value,ok", [
    ("pre_filter_cap", 0, False), ("pre_filter_cap", 63, True), ("pre_filter_cap", 64, False),
    ("pre_filter_size", 4, False), ("pre_filter_size", 6, False), ("pre_filter_size", 5, True),
    ("block_size", 4, False), ("block_size", 10, False), ("block_size", 481, False),
    ("block_size", 255, True), ("num_disparities", 72, False), ("texture_threshold", -1, False),
    ("uniqueness_ratio", -1, False), ("pre_filter_type", 2, False)])
def test_bm_validation_rules(mvsv, field, value, ok):
    """StereoBMImpl::compute's CV_Error checks ([OpenCV] stereobm.cpp), SURVEY §8(b)."""
    from mvstereovision3_amd import _lib
    b = mvsv.StereoBM.create(64, 9)
    setattr(b._params, field, value)
    rc = _lib.lib().mvsv_bm_validate(ctypes.byref(b._params), 640, 480)
    assert (rc == 0) == ok


def test_load_sgbm_yml(mvsv):
    """Disparity::loadSGBMParameters (src/disparity.cpp:60-108) on configs/sgbm.yml."""
    m = mvsv.StereoSGBM.create(0, 0, 0, 8 * 0 * 0, 32 * 0 * 0)  # trgt/mean_test.cpp:233-237
    para = mvsv.sgbmParameters()
    assert mvsv.Disparity.loadSGBMParameters(os.path.join(CONFIGS, "sgbm.yml"), m, para)
    assert (para.minDisp, para.numDisp, para.blockSize, para.disp12MaxDiff, para.preFilterCap,
            para.uniquenessRatio, para.speckleWindowSize, para.speckleRange,
            para.disparityMode) == (1, 128, 13, 0, 0, 0, 150, 2, 0)
    p = m.params()
    # the eight setters + mode; P1/P2 untouched (effective 2 / 5 in OpenCV)
    assert p["min_disparity"] == 1 and p["num_disparities"] == 128 and p["block_size"] == 13
    assert p["speckle_window_size"] == 150 and p["speckle_range"] == 2 and p["mode"] == 0
    assert p["p1"] == 0 and p["p2"] == 0


def test_load_sgbm_backup_and_mode(mvsv, tmp_path):
    m = mvsv.StereoSGBM.create()
    para = mvsv.sgbmParameters()
    assert mvsv.Disparity.loadSGBMParameters(os.path.join(CONFIGS, "sgbm.yml.bak"), m, para)
    assert para.numDisp == 144 and para.blockSize == 7
    f = tmp_path / "hh.yml"
    f.write_text("%YAML:1.0\nnumDisp: 64\nblockSize: 5\nspeckleWindowSize: 0\n"
                 "speckleWindowRange: 0\nmode: 1\n")
    assert mvsv.Disparity.loadSGBMParameters(str(f), m, para)
    assert m.getMode() == mvsv.MODE_HH and para.minDisp == 0  # missing key -> 0


def test_load_sgbm_failures(mvsv, tmp_path):
    m = mvsv.StereoSGBM.create()
    para = mvsv.sgbmParameters()
    assert not mvsv.Disparity.loadSGBMParameters(str(tmp_path / "missing.yml"), m, para)
    f = tmp_path / "partial.yml"
    f.write_text("%YAML:1.0\nnumDisp: 64\nblockSize: 5\nspeckleWindowSize: 10\n")
    assert not mvsv.Disparity.loadSGBMParameters(str(f), m, para)  # speckleWindowRange missing


def test_load_bm_yml(mvsv):
    b = mvsv.StereoBM.create(16, 9)
    assert mvsv.Disparity.loadBMParameters(os.path.join(CONFIGS, "bm.yml"), b)
    p = b.params()
    assert (p["num_disparities"], p["block_size"], p["pre_filter_cap"], p["pre_filter_size"],
            p["uniqueness_ratio"], p["texture_threshold"]) == (80, 21, 2, 51, 0, 30)
    assert mvsv.Disparity.loadBMParameters(os.path.join(CONFIGS, "bm.yml.bak"), b)
    assert b.getNumDisparities() == 128


def _pcg32_stream(seed, n):
    state = (seed * 2 + 1) & (2**64 - 1)
    inc = 0xda3e39cb94b95bdb
    out = []
    for _ in range(n):
        old = state
        state = (old * 6364136223846793005 + inc) & (2**64 - 1)
        xs = (((old >> 18) ^ old) >> 27) & 0xffffffff
        rot = old >> 59
        out.append(((xs >> rot) | (xs << ((-rot) & 31))) & 0xffffffff)
    return out


def test_synth_pair_matches_spec(mvsv):
    """SURVEY.md §8(d) generator restated in numpy on a small frame."""
    W, H, minD, D, seed = 24, 12, 0, 16, 0x5EED0000
    L, R = mvsv.synth_pair(seed, W, H, minD, D)
    st = _pcg32_stream(seed, 2 * W * H)
    noise = (np.array(st[:W * H], np.uint64) >> 24).astype(np.int64).reshape(H, W)
    P = np.pad(noise, 1, mode="edge")
    s = sum(P[dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3))
    L2 = ((2 * s + 9) // 18).astype(np.uint8)
    assert np.array_equal(L, L2)
    rect = int(np.floor(0.6 * D + 0.5))
    R2 = np.zeros_like(L2)
    k = W * H
    for y in range(H):
        for x in range(W):
            inside = W // 3 <= x < 2 * W // 3 and H // 3 <= y < 2 * H // 3
            d = rect if inside else int(np.floor(D / 8 + (D / 4) * y / H + 0.5))
            d = min(max(d, minD), minD + D - 1)
            v = int(L2[y, min(max(x + d, 0), W - 1)]) + int(st[k] % 3) - 1
            k += 1
            R2[y, x] = min(max(v, 0), 255)
    assert np.array_equal(R, R2)


def test_synth_pair_deterministic(mvsv):
    a = mvsv.synth_pair(1, 64, 48, 0, 16)
    b = mvsv.synth_pair(1, 64, 48, 0, 16)
    c = mvsv.synth_pair(2, 64, 48, 0, 16)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert not np.array_equal(a[0], c[0])


def test_no_device_fails_loudly(mvsv):
    """Without a HIP device the product path raises; there is no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from mvstereovision3_amd import _lib
    h = ctypes.c_void_p()
    assert _lib.lib().mvsv_create(ctypes.byref(h), 0) == _lib.MVSV_E_NODEV
    L, R = mvsv.synth_pair(0, 64, 48, 0, 16)
    with pytest.raises(mvsv.MvsvError):
        mvsv.StereoSGBM.create(0, 16, 5).compute(L, R)
