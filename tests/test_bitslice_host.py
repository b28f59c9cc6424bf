"""Host check of the bit-sliced SGM arithmetic (round 5): tests/cpp/bitslice_check.cpp
runs mvsv_bitslice.hpp's helpers against their scalar definitions, whole scanlines
of the lane-pair and lane-quad direction steps the bit-sliced kernels run
(mvsv_bsgm.hip) against OpenCV 3.4's recurrence on unclamped costs (SURVEY
Appendix A.4), the grouped plane layouts, and the cost kernel's 32 x 32 lane
transpose against its definition."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bitslice_arithmetic(tmp_path):
    exe = tmp_path / "bsc"
    subprocess.run(["g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "bitslice_check.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "bitslice checks: 0 failures" in r.stdout
