"""Regenerate tests/golden/fixtures.npz (small input/expected-output vectors).

No golden vectors exist in the reference for this path (SURVEY.md §8(c):
parity unpinned; OpenCV absent).  These fixtures are produced by the C oracle
(oracle/mvsv_oracle.c, OpenCV 3.4 restatement) and are only written when the
independent numpy restatement (oracle/twin.py) agrees bit for bit.  They pin
the checker against regressions and give the GPU tests oracle-free vectors.

Inputs are the deterministic synthetic pairs of SURVEY.md §8(d)
(libmvsv's mvsv_synth_pair; the generator itself is checked against a numpy
PCG32 in tests/test_abi.py).

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from mvstereovision3_amd import synth_pair  # noqa: E402
from oracle import pyoracle, twin  # noqa: E402

SEED0 = 0x5EED0000

SGBM_CASES = [
    # name, (W, H, minD, D), params (OpenCV create order) , variant
    ("sgbm_yml_mode0", (160, 96, 1, 32),
     dict(min_disparity=1, num_disparities=32, block_size=13, p1=0, p2=0, disp12_max_diff=0,
          pre_filter_cap=0, uniqueness_ratio=0, speckle_window_size=150, speckle_range=2, mode=0), 0),
    ("sgbm_yml_hh", (160, 96, 1, 32),
     dict(min_disparity=1, num_disparities=32, block_size=13, p1=0, p2=0, disp12_max_diff=0,
          pre_filter_cap=0, uniqueness_ratio=0, speckle_window_size=150, speckle_range=2, mode=1), 0),
    ("live_disparity", (128, 80, 0, 32),
     dict(min_disparity=0, num_disparities=32, block_size=9, p1=648, p2=2592, disp12_max_diff=0,
          pre_filter_cap=0, uniqueness_ratio=0, speckle_window_size=0, speckle_range=0, mode=0), 0),
    ("capture_disparity", (96, 64, 0, 16),
     dict(min_disparity=0, num_disparities=16, block_size=5, p1=200, p2=800, disp12_max_diff=0,
          pre_filter_cap=0, uniqueness_ratio=0, speckle_window_size=0, speckle_range=0, mode=0), 0),
    ("sgbm_uniq_neg_mind", (120, 72, -4, 32),
     dict(min_disparity=-4, num_disparities=32, block_size=7, p1=72, p2=288, disp12_max_diff=2,
          pre_filter_cap=31, uniqueness_ratio=10, speckle_window_size=30, speckle_range=4, mode=1), 0),
    ("sgbm_variant_4x", (120, 72, 0, 32),
     dict(min_disparity=0, num_disparities=32, block_size=5, p1=0, p2=0, disp12_max_diff=1,
          pre_filter_cap=15, uniqueness_ratio=5, speckle_window_size=0, speckle_range=0, mode=0), 3),
]

BM_CASES = [
    ("bm_defaults_64_9", (160, 96, 0, 64),
     dict(pre_filter_type=1, pre_filter_size=9, pre_filter_cap=31, block_size=9, min_disparity=0,
          num_disparities=64, texture_threshold=10, uniqueness_ratio=15, speckle_window_size=0,
          speckle_range=0, disp12_max_diff=-1)),
    ("bm_yml", (200, 96, 0, 80),
     dict(pre_filter_type=1, pre_filter_size=51, pre_filter_cap=2, block_size=21, min_disparity=0,
          num_disparities=80, texture_threshold=30, uniqueness_ratio=0, speckle_window_size=0,
          speckle_range=0, disp12_max_diff=-1)),
    ("bm_validate_speckle", (128, 80, 0, 32),
     dict(pre_filter_type=1, pre_filter_size=9, pre_filter_cap=31, block_size=7, min_disparity=0,
          num_disparities=32, texture_threshold=10, uniqueness_ratio=5, speckle_window_size=40,
          speckle_range=16, disp12_max_diff=1)),
]


def main():
    arrays, meta = {}, {"sgbm": [], "bm": []}
    for k, (name, (W, H, mind, D), p, variant) in enumerate(SGBM_CASES):
        L, R = synth_pair(SEED0 + 100 + k, W, H, mind, D)
        want = pyoracle.sgbm(L, R, p, flags=variant)
        assert np.array_equal(want, twin.sgbm_compute(L, R, p, variant)), name
        arrays[f"{name}_L"], arrays[f"{name}_R"], arrays[f"{name}_out"] = L, R, want
        meta["sgbm"].append({"name": name, "params": p, "variant": variant})
    for k, (name, (W, H, mind, D), p) in enumerate(BM_CASES):
        L, R = synth_pair(SEED0 + 200 + k, W, H, mind, D)
        want = pyoracle.bm(L, R, p)
        assert np.array_equal(want, twin.bm_compute(L, R, p)), name
        arrays[f"{name}_L"], arrays[f"{name}_R"], arrays[f"{name}_out"] = L, R, want
        meta["bm"].append({"name": name, "params": p})
    # cost volume of a small case (quirk rows / column included)
    L, R = synth_pair(SEED0 + 300, 64, 24, 0, 16)
    p = dict(SGBM_CASES[1][2], min_disparity=0, num_disparities=16, block_size=5)
    Cv = pyoracle.sgbm_cost_volume(L, R, p)
    assert np.array_equal(Cv, twin.sgbm_cost_volume(L, R, p))
    arrays["costvol_L"], arrays["costvol_R"], arrays["costvol_C"] = L, R, Cv
    meta["costvol_params"] = p
    # post-pass on a disparity map: median, speckle, 9x9 mean grid
    d = arrays["sgbm_yml_hh_out"]
    arrays["post_in"] = d
    arrays["post_median"] = pyoracle.median3x3(d)
    arrays["post_speckle"] = pyoracle.filter_speckles(d, 0, 20, 16)
    arrays["post_grid"] = pyoracle.mean_disparity_grid(d)
    assert np.array_equal(arrays["post_median"], twin.median3x3(d))
    assert np.array_equal(arrays["post_speckle"], twin.filter_speckles(d, 0, 20, 16))
    assert np.array_equal(arrays["post_grid"], twin.mean_disparity_grid(d))
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures.npz")
    np.savez_compressed(out, **arrays)
    with open(os.path.join(os.path.dirname(out), "fixtures.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
