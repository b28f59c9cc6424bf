"""MeanDisparityDetection mirror: host decisions.

Reference: src/MeanDisparityDetection.cpp:71-266 (init / build / detectObstacles),
inc/Subimage.h:17-47, trgt/mean_test.cpp:80-106 (createDMapROIS).  The 9x9 means
are supplied directly here (their GPU kernel is checked in test_gpu_parity.py);
these tests pin the host logic against a numpy restatement.
"""
import json
import os

import numpy as np

from conftest import GOLDEN

Q_REF = np.array(json.load(open(os.path.join(GOLDEN, "q_matrix.json")))["Q"], np.float32)


def test_positions_map_is_the_reference_table(mvsv):
    from mvstereovision3_amd.detection import POSITIONS
    assert 10 not in POSITIONS and len(POSITIONS) == 81  # the reference skips key 10
    assert POSITIONS[9] == "TOP - 0" and POSITIONS[11] == "TOP - 1" and POSITIONS[18] == "TOP - 8"
    assert POSITIONS[37] == "CENTER - 0" and POSITIONS[81] == "BOTTOM RIGHT - 8"


def test_init_tiles_and_disparity_range(mvsv):
    m = mvsv.MeanDisparityDetection()
    m.init((480, 752 - 64), Q_REF, 0.1, 1.5)
    tiles = m.getSubimageVec()
    assert len(tiles) == 81
    dx, dy = (752 - 64) // 9, 480 // 9
    assert tiles[10].tl == (dx, dy) and tiles[10].br == (2 * dx, 2 * dy)
    assert tiles[10].roi_center == (dx + dx // 2, dy + dy // 2)
    q = Q_REF.reshape(4, 4)
    for z, got in ((100.0, m.mRangeDisparity[0]), (1500.0, m.mRangeDisparity[1])):
        disp = np.float32((np.float32(q[2, 3]) - np.float32(z) * np.float32(q[3, 3])) /
                          (np.float32(z) * np.float32(q[3, 2])))
        assert np.float32(got) == np.float32(disp * np.float32(16))


def test_create_dmap_rois(mvsv):
    roi_u, roi_b = mvsv.create_dmap_rois((960, 1280), 256)
    assert roi_u == (128, 0, 1280, 960) and roi_b == (64, 0, 640, 480)


def test_detect_obstacles_mean_value(mvsv, tmp_path):
    m = mvsv.MeanDisparityDetection(pcl_dir=str(tmp_path))
    m.init((480, 688), Q_REF, 0.1, 1.5)
    lo, hi = m.mRangeDisparity  # lo = far (large disparity), hi = near bound
    means = np.zeros(81, np.float32)
    means[[3, 40, 77]] = [np.float32(hi) + 16, np.float32(lo) - 1, np.float32(lo) + 10]
    dmap = np.full((480, 688), 200, np.int16)
    m.build(dmap, 0, m.MEAN_VALUE, means=means)
    assert m.getMeanMap() == [float(v) for v in means]
    m.detectObstacles()
    found = [s.tl for s in m.getFoundObstacles()]
    want = [m.getSubimageVec()[i].tl for i in range(81)
            if np.float32(means[i]) < np.float32(lo) and np.float32(means[i]) > np.float32(hi)]
    assert found == want and len(found) == 2
    assert (tmp_path / "pcl_0000.ply").exists() and m.getObstacleCounter() == 1


def test_mean_distance_falls_through_to_mean_value(mvsv):
    from mvstereovision3_amd.utility import Utility, dMapValues
    m = mvsv.MeanDisparityDetection()
    m.init((480, 688), Q_REF, 0.1, 1.5)
    means = np.arange(81, dtype=np.float32) * 7
    m.build(np.zeros((480, 688), np.int16), 0, m.MEAN_DISTANCE, means=means)
    assert m.mDetectionMode == m.MEAN_VALUE  # no break in the reference's switch
    assert len(m.getMeanMap()) == 81
    s = m.getSubimageVec()[5]
    assert m.getMeanDistanceMap()[5] == Utility.calcDistance(
        dMapValues(means[5], s.roi_center[0], s.roi_center[1]), Q_REF, 0)


def test_detect_obstacles_batched_points_match_per_tile(mvsv):
    """detectObstacles' one native call for all found tiles (mvsv_calc_coordinates)
    gives the points of the reference's per-tile Utility::calcCoordinate loop
    (src/MeanDisparityDetection.cpp:228-240), bit for bit, on many found tiles."""
    from mvstereovision3_amd.utility import Utility, dMapValues
    m = mvsv.MeanDisparityDetection()
    m.init((960, 1152), Q_REF, 0.1, 1.5)
    lo, hi = (np.float32(v) for v in m.mRangeDisparity)
    rng = np.random.default_rng(77)
    means = rng.uniform(float(hi) - 50, float(lo) + 50, 81).astype(np.float32)
    means[:4] = [hi, lo, np.nextafter(hi, np.float32(1e9)), np.nextafter(lo, np.float32(-1e9))]
    m.build(np.zeros((960, 1152), np.int16), 0, m.MEAN_VALUE, means=means)
    m.detectObstacles(write_pcl=False)
    want_tiles, want_pts = [], []
    for i, s in enumerate(m.getSubimageVec()):
        if means[i] < lo and means[i] > hi:
            want_tiles.append(s.tl)
            want_pts.append(Utility.calcCoordinate(dMapValues(means[i], *s.roi_center), m.mQ_32F))
    assert [s.tl for s in m.getFoundObstacles()] == want_tiles and len(want_tiles) > 20
    assert len(m.mFoundPoints) == len(want_pts)
    for got, want in zip(m.mFoundPoints, want_pts):
        assert got.dtype == np.float32 and np.array_equal(got.view(np.uint32), want.view(np.uint32))
