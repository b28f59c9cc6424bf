"""AddressSanitizer + UBSan build of the host code (SURVEY.md §5 "Race detection /
sanitizers"): the HIP-free translation unit of libmvsv (mvsv_io.cpp: YAML readers,
calibration files, stereoRectify, undistort maps, PLY writer, synthetic pairs),
the frame stream's slot bookkeeping (mvsv_ring.hpp, randomized push / pop /
set_batch sequences) and the CPU oracle, driven by tests/cpp/sanitize_driver.cpp.
Any sanitizer report aborts the driver (-fno-sanitize-recover=all)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
       "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None,
                    reason="needs gcc/g++")
def test_host_code_under_asan_ubsan(tmp_path):
    obj = tmp_path / "oracle.o"
    subprocess.run(["gcc", "-std=c99", *SAN, "-c", os.path.join(ROOT, "oracle", "mvsv_oracle.c"),
                    "-o", str(obj)], check=True)
    exe = tmp_path / "sanitize_driver"
    subprocess.run(["g++", "-std=c++17", *SAN,
                    os.path.join(ROOT, "tests", "cpp", "sanitize_driver.cpp"),
                    os.path.join(ROOT, "mvstereovision3_amd", "csrc", "mvsv_io.cpp"), str(obj),
                    "-o", str(exe), "-lm"], check=True)
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1"
    work = tmp_path / "work"
    work.mkdir()
    r = subprocess.run([str(exe), os.path.join(ROOT, "tests", "golden"), str(work)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "0 failures" in r.stdout
