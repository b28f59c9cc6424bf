#!/usr/bin/env python3
"""BASELINE config 5: a camera-loop stream through the frame pipeline.

liveDisparity-style matcher create(0, 256, 9, 8*81, 32*81) (MODE_SGBM, no speckle)
on 1280x960 synthetic rectified pairs, followed by MeanDisparityDetection
(build(MEAN_VALUE) on the createDMapROIS work ROI x in [128, W), detectObstacles)
per frame -- the loop of trgt/mean_test.cpp:258-318 without its worker thread.
Host frames go in, int16 maps and the 81 tile means come back (PCIe included);
`depth` frames are in flight, computed `batch` at a time.  Also reports the device-resident rate of the same
matcher on a batch of 8 frames.  Not the headline metric (bench.py is).

    python tools/bench_stream.py [--frames 300] [--depth 24] [--batch 8] [--inflight 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stream_measure(mvsv, W=1280, H=960, frames=300, depth=24, batch=8, inflight=2, pop="view",
                   host_probe="full", device_steps=10):
    """The config-5 stream (liveDisparity matcher + MeanDisparityDetection post-pass
    on every frame, host frames in / maps and means out) -> one result dict."""
    import numpy as np
    import torch

    D = 256
    m = mvsv.StereoSGBM.create(0, D, 9, 8 * 81, 32 * 81)  # trgt/liveDisparity.cpp:61
    q = json.load(open(os.path.join(ROOT, "tests", "golden", "q_matrix.json")))["Q"]
    Q = np.array(q, np.float32).reshape(4, 4)
    Q[0, 3] *= 2  # afterCalibrationParameters.yml is for 752x480: x2 for 1280x960-class sensors
    Q[1, 3] *= 2
    Q[2, 3] *= 2
    roi_u, _ = mvsv.create_dmap_rois((H, W), D)
    det = mvsv.MeanDisparityDetection()
    det.init((roi_u[3] - roi_u[1], roi_u[2] - roi_u[0]), Q, 0.1, 1.5)
    uniq = [mvsv.synth_pair(0x5EED0000 + i, W, H, 0, D) for i in range(8)]

    st = mvsv.DisparityStream(m, W, H, depth=depth, grid_roi=roi_u, batch=batch, inflight=inflight)
    found = 0
    host = {"push": 0.0, "pop": 0.0, "post": 0.0}

    def consume():
        nonlocal found
        t = time.perf_counter()
        if host_probe == "no-copy":
            st.pop(copy_map=False)
        else:
            d, means = st.pop(copy_map="view" if pop == "view" else True)
        t2 = time.perf_counter()
        if host_probe == "full":
            det.build(d, 0, det.MEAN_VALUE, means=means)
            det.detectObstacles(write_pcl=False)
            found += len(det.getFoundObstacles())
        host["pop"] += t2 - t
        host["post"] += time.perf_counter() - t2

    for i in range(depth):  # warm-up
        st.push(*uniq[i % 8])
    while st.pending():
        consume()
    host = dict.fromkeys(host, 0.0)
    t0 = time.perf_counter()
    for i in range(frames):
        if st.pending() == depth:
            consume()
        t = time.perf_counter()
        st.push(*uniq[i % 8])
        host["push"] += time.perf_counter() - t
    while st.pending():
        consume()
    wall = time.perf_counter() - t0
    st.close()

    # device-resident rate of the same matcher + the mean grid (8-frame batch in HBM)
    dev = torch.device("cuda", 0)
    Lt = torch.from_numpy(np.stack([u[0] for u in uniq])).to(dev)
    Rt = torch.from_numpy(np.stack([u[1] for u in uniq])).to(dev)
    out = torch.empty((8, H, W), dtype=torch.int16, device=dev)
    for _ in range(2):
        m.compute(Lt, Rt, out)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(device_steps):
        m.compute(Lt, Rt, out)
        mvsv.mean_disparity_grid(out[:, roi_u[1]:roi_u[3], roi_u[0]:roi_u[2]])
    torch.cuda.synchronize()
    dwall = time.perf_counter() - t1
    return {
        "workload": f"config5_stream_{W}x{H}_d{D}_mode_sgbm",
        "frames": frames, "depth": depth, "batch": batch, "inflight": inflight,
        "host_probe": host_probe, "pop": pop,
        "stream_fps": round(frames / wall, 2),
        "stream_mpix_s": round(frames * W * H / wall / 1e6, 2),
        "stream_ms_per_frame": round(wall / frames * 1e3, 3),
        "device_resident_mpix_s": round(8 * device_steps * W * H / dwall / 1e6, 2),
        "device_resident_ms_per_frame": round(dwall / (8 * device_steps) * 1e3, 3),
        "obstacle_tiles_found": found,
        "host_ms_per_frame": {k: round(v / frames * 1e3, 3) for k, v in host.items()},
        "note": "stream = host frames in, int16 map + 81 means out (PCIe incl.); "
                "post-pass = MeanDisparityDetection build(MEAN_VALUE) + detectObstacles",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--depth", type=int, default=24)
    ap.add_argument("--batch", type=int, default=8, help="frames per SGBM launch (mvsv_stream_set_batch)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="launches computed concurrently (mvsv_stream_set_inflight)")
    ap.add_argument("--pop", choices=["view", "copy"], default="view",
                    help="map delivery: a read-only view of the pinned slot (mvsv_stream_pop_view) "
                         "or a copy into a fresh array (mvsv_stream_pop)")
    ap.add_argument("--host-probe", choices=["full", "no-post", "no-copy"], default="full",
                    help="diagnostics: skip the detection post-pass, or also the map copy of pop")
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=960)
    a = ap.parse_args()
    import mvstereovision3_amd as mvsv
    print(json.dumps(stream_measure(mvsv, a.width, a.height, a.frames, a.depth, a.batch, a.inflight, a.pop,
                                    a.host_probe)))


if __name__ == "__main__":
    main()
