"""The C++ drop-in (include/mvsv_disparity.hpp) compiled with g++ against the
C ABI, exercising the reference's call pattern (src/disparity.cpp:6-108,
trgt/mean_test.cpp:233-241)."""
import os
import subprocess

import numpy as np
import pytest

from tests.conftest import CONFIGS, ROOT


@pytest.fixture(scope="module")
def adapter_bin(tmp_path_factory):
    from mvstereovision3_amd import _lib
    _lib.lib()
    out = str(tmp_path_factory.mktemp("cpp") / "adapter_check")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "adapter_check.cpp"),
                    "-L", libdir, "-lmvsv", f"-Wl,-rpath,{libdir}", "-o", out], check=True)
    return out


def test_cpp_adapter_cpu(adapter_bin):
    r = subprocess.run([adapter_bin, "cpu", CONFIGS], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "cpu ok" in r.stdout


@pytest.mark.gpu
def test_cpp_adapter_gpu(adapter_bin, tmp_path, gpu, oracle):
    import mvstereovision3_amd as mvsv
    path = str(tmp_path / "out.bin")
    r = subprocess.run([adapter_bin, "gpu", CONFIGS, path], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = np.fromfile(path, dtype=np.int16)
    w, h = 320, 160
    d1, d2 = raw[: w * h].reshape(h, w), raw[w * h:].reshape(h, w)
    L, R = mvsv.synth_pair(0x5EED0000 + 77, 400, 200, 1, 128)
    L, R = L[8:168, 16:336], R[8:168, 16:336]
    p = dict(min_disparity=1, num_disparities=128, block_size=13, p1=0, p2=0, disp12_max_diff=0,
             pre_filter_cap=0, uniqueness_ratio=0, speckle_window_size=150, speckle_range=2,
             mode=0)
    assert np.array_equal(d1, oracle.sgbm(L, R, p))
    b = mvsv.StereoBM.create(64, 9).params()
    assert np.array_equal(d2, oracle.bm(L, R, b))


@pytest.fixture(scope="module")
def detection_bin(tmp_path_factory):
    from mvstereovision3_amd import _lib
    _lib.lib()
    out = str(tmp_path_factory.mktemp("cppdet") / "detection_check")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-Wno-implicit-fallthrough",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "detection_check.cpp"),
                    "-L", libdir, "-lmvsv", f"-Wl,-rpath,{libdir}", "-o", out], check=True)
    return out


def test_cpp_detection_cpu(detection_bin, tmp_path):
    r = subprocess.run([detection_bin, "cpu", str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpu ok" in r.stdout
    assert (tmp_path / "two.ply").read_text().startswith("ply\nformat ascii 1.0\ncomment author: Hagen Hiller")


@pytest.mark.gpu
def test_cpp_detection_gpu(detection_bin, tmp_path, gpu):
    r = subprocess.run([detection_bin, "gpu", str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu ok" in r.stdout and (tmp_path / "cloud.ply").exists()
