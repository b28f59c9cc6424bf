"""The C++ Stereosystem mirror (include/mvsv_stereosystem.hpp) compiled with g++
against the C ABI: calibration files, stereoRectify (pinned by the reference's
own afterCalibrationParameters.yml and parameters/*/*.yml), and both
getRectifiedImagepair overloads (src/Stereosystem.cpp:193-315) on the GPU,
checked against the oracle's remap + crop (+ resize)."""
import os
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

CAL = os.path.join(ROOT, "tests", "golden", "calib")


@pytest.fixture(scope="module")
def stereosystem_bin(tmp_path_factory):
    from mvstereovision3_amd import _lib
    _lib.lib()
    out = str(tmp_path_factory.mktemp("cppss") / "stereosystem_check")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "stereosystem_check.cpp"),
                    "-L", libdir, "-lmvsv", f"-Wl,-rpath,{libdir}", "-o", out], check=True)
    return out


def test_cpp_stereosystem_cpu(stereosystem_bin, tmp_path):
    r = subprocess.run([stereosystem_bin, "cpu", CAL, str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpu ok" in r.stdout
    assert "STEREOSYSTEM\tRectification successfully initialized!" in r.stderr


def _load(path):
    with open(path, "rb") as f:
        h, w = map(int, f.readline().split())
        return np.frombuffer(f.read(), np.uint8).reshape(h, w)


@pytest.mark.gpu
def test_cpp_stereosystem_gpu(stereosystem_bin, tmp_path, gpu, oracle):
    from mvstereovision3_amd import calibration as calib
    r = subprocess.run([stereosystem_bin, "gpu", CAL, str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu ok" in r.stdout
    # the same rectification state through the Python mirror (same host maps)
    s = calib.Stereosystem(376, 240, binning=True)
    assert s.loadIntrinsic(os.path.join(CAL, "baseline_small", "intrinsic.yml"))
    assert s.loadExtrinisic(os.path.join(CAL, "baseline_small", "extrinsic.yml"))
    assert s.initRectification()
    x0, y0, x1, y1 = s.mDisplayROI
    want = {}
    for side, k in (("l", 0), ("r", 1)):
        raw = _load(tmp_path / f"raw_{side}.bin")
        full = oracle.remap_linear(raw, s.mMap1[k], s.mMap2[k])
        want[side] = full[y0:y1, x0:x1]
        assert np.array_equal(_load(tmp_path / f"init_{side}.bin"), want[side]), "init call: crop only"
        assert np.array_equal(_load(tmp_path / f"rect_{side}.bin"), want[side])
        for f in ("0.5", "0.75", "1.5", "0.3"):
            got = _load(tmp_path / f"res_{f}_{side}.bin")
            ff = float(np.float32(float(f)))
            assert np.array_equal(got, oracle.resize_linear(want[side], ff, ff)), f"factor {f} {side}"
