"""BASELINE config 5 at full size: the liveDisparity-style stream.

1280x960 pairs, StereoSGBM::create(0, 256, 9, 8*9*9, 32*9*9) -- the matcher of
trgt/liveDisparity.cpp:61 (MODE_SGBM, no speckle filter), computed through
DisparityStream (the mvsv_stream C ABI; frame-batch launches of 8) with the
MeanDisparityDetection 9x9 grid on the work ROI of createDMapROIS
(trgt/mean_test.cpp:80-106: x in [D/2, W)), src/MeanDisparityDetection.cpp:159-206.
Every map and its 81 means must equal the oracle bit for bit.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED0 = 0x5EED0000
W, H, D = 1280, 960, 256


def test_config5_stream_full_size(gpu, mvsv, oracle):
    m = mvsv.StereoSGBM.create(0, D, 9, 8 * 9 * 9, 32 * 9 * 9)  # trgt/liveDisparity.cpp:61
    roi_u, _ = mvsv.create_dmap_rois((H, W), D)
    assert roi_u == (128, 0, W, H)
    frames = [mvsv.synth_pair(SEED0 + 500 + i, W, H, 0, D) for i in range(3)]
    st = mvsv.DisparityStream(m, W, H, depth=8, grid_roi=roi_u, batch=8)
    for L, R in frames:
        st.push(L, R)
    got = [st.pop() for _ in frames]  # the first pop launches the partial group of 3
    st.close()

    p = dict(m.params())
    p.pop("variant")
    with ThreadPoolExecutor(len(frames)) as ex:  # the oracle releases the GIL
        want = list(ex.map(lambda f: oracle.sgbm(f[0], f[1], p), frames))
    x0, y0, x1, y1 = roi_u
    for i, ((d, means), w) in enumerate(zip(got, want)):
        bad = np.argwhere(d != w)
        assert bad.size == 0, f"frame {i}: {len(bad)} mismatches, first {bad[:5].tolist()}"
        wm = oracle.mean_disparity_grid(np.ascontiguousarray(w[y0:y1, x0:x1]))
        assert np.array_equal(means, wm), f"frame {i}: means differ"
        # the synthetic field is known: most of the map is matched (not INVALID)
        assert (w > 0).mean() > 0.5


def test_config5_detection_on_stream_means(gpu, mvsv, oracle):
    """The obstacle pass of trgt/mean_test.cpp:258-318 on GPU means equals the
    same pass on oracle means (MeanDisparityDetection::detectObstacles)."""
    m = mvsv.StereoSGBM.create(0, D, 9, 8 * 9 * 9, 32 * 9 * 9)
    roi_u, _ = mvsv.create_dmap_rois((H, W), D)
    L, R = mvsv.synth_pair(SEED0 + 510, W, H, 0, D)
    st = mvsv.DisparityStream(m, W, H, depth=2, grid_roi=roi_u)
    st.push(L, R)
    d, means = st.pop()
    st.close()
    x0, y0, x1, y1 = roi_u
    work = np.ascontiguousarray(d[y0:y1, x0:x1])
    Q = np.array([[1, 0, 0, -640], [0, 1, 0, -480], [0, 0, 0, 1400], [0, 0, 1 / 0.12, 0]],
                 np.float32).reshape(16)
    det = mvsv.MeanDisparityDetection()
    det.init(work.shape, Q, 0.1, 1.5)
    det.build(work, 0, det.MEAN_VALUE, means=means)
    det.detectObstacles(write_pcl=False)
    ref = mvsv.MeanDisparityDetection()
    ref.init(work.shape, Q, 0.1, 1.5)
    ref.build(work, 0, ref.MEAN_VALUE, means=oracle.mean_disparity_grid(work))
    ref.detectObstacles(write_pcl=False)
    assert det.getMeanMap() == ref.getMeanMap()
    assert [s.tl for s in det.getFoundObstacles()] == [s.tl for s in ref.getFoundObstacles()]
