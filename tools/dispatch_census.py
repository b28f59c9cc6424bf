#!/usr/bin/env python3
"""Which kernel instances each BASELINE config and reference call site dispatches.

    python tools/dispatch_census.py CONFIG      (run under rocprofv3 --kernel-trace)
    python tools/dispatch_census.py --collect DIR OUT.json
        (DIR/<config>/run_kernel_trace.csv -> {config: {kernel name: scratch bytes}})

CONFIG: c1 (StereoBM configs/bm.yml 640x480), c2 (StereoBM(64, 9) 640x480),
c3m0 / c3m1 (configs/sgbm.yml 640x480, mode 0 / 1), c4 (sgbm.yml MODE_HH
1280x960), c4m0 (sgbm.yml mode 0 1280x960), c5 (liveDisparity create(0, 256, 9,
648, 2592) 1280x960 and its stream), live64 (liveDisparity's default
create(0, 64, 9, 648, 2592), trgt/liveDisparity.cpp:19-20,61), capture
(captureDisparity create(0, 16, 5, 200, 800), trgt/captureDisparity.cpp:24-25,196).
Each runs batches of 1, 2 and 8 frames (the launch-shape choices differ).
tests/test_kernel_scratch.py checks the recorded instances for scratch.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CFG = os.path.join(ROOT, "tests", "golden", "configs")
CONFIGS = ["c1", "c2", "c3m0", "c3m1", "c4", "c4m0", "c5", "live64", "capture"]


def run(name):
    import numpy as np
    import torch
    import mvstereovision3_amd as mvsv
    dev = torch.device("cuda", 0)

    def sgbm_yml(mode):
        m = mvsv.StereoSGBM.create(0, 0, 0, 0, 0)
        assert mvsv.Disparity.loadSGBMParameters(os.path.join(CFG, "sgbm.yml"), m, mvsv.sgbmParameters())
        m.setMode(mode)
        return m

    if name == "c1":
        m, W, H, D, minD = mvsv.StereoBM.create(0, 21), 640, 480, 80, 0
        assert mvsv.Disparity.loadBMParameters(os.path.join(CFG, "bm.yml"), m)
    elif name == "c2":
        m, W, H, D, minD = mvsv.StereoBM.create(64, 9), 640, 480, 64, 0
    elif name in ("c3m0", "c3m1"):
        m, W, H, D, minD = sgbm_yml(int(name[-1])), 640, 480, 128, 1
    elif name in ("c4", "c4m0"):
        m, W, H, D, minD = sgbm_yml(1 if name == "c4" else 0), 1280, 960, 128, 1
    elif name == "c5":
        m, W, H, D, minD = mvsv.StereoSGBM.create(0, 256, 9, 648, 2592), 1280, 960, 256, 0
    elif name == "live64":
        m, W, H, D, minD = mvsv.StereoSGBM.create(0, 64, 9, 648, 2592), 1280, 960, 64, 0
    elif name == "capture":
        m, W, H, D, minD = mvsv.StereoSGBM.create(0, 16, 5, 200, 800), 640, 480, 16, 0
    else:
        raise SystemExit(f"unknown config {name}")
    pairs = [mvsv.synth_pair(0x5EED0000 + i, W, H, minD, D) for i in range(8)]
    for n in (1, 2, 8):
        L = torch.from_numpy(np.stack([p[0] for p in pairs[:n]])).to(dev)
        R = torch.from_numpy(np.stack([p[1] for p in pairs[:n]])).to(dev)
        out = torch.empty((n, H, W), dtype=torch.int16, device=dev)
        m.compute(L, R, out)
    if name == "c5":
        from tools.bench_stream import stream_measure
        stream_measure(mvsv, frames=16, depth=8, batch=8, inflight=2, device_steps=1)
    torch.cuda.synchronize()
    mvsv.synchronize()


def collect(d, out):
    res = {}
    for name in CONFIGS:
        files = glob.glob(os.path.join(d, name, "**", "*kernel_trace.csv"), recursive=True)
        ks = {}
        for f in files:
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if k.startswith("__amd_rocclr") or "at::" in k or "elementwise" in k.lower():
                    continue
                ks[k] = max(ks.get(k, 0), int(r.get("Scratch_Size") or 0))
        res[name] = ks
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for name, ks in res.items():
        bad = {k: v for k, v in ks.items() if v}
        print(name, len(ks), "kernels,", len(bad), "with scratch", *[f"\n   {v:5d} B {k[:110]}" for k, v in bad.items()])


if __name__ == "__main__":
    if sys.argv[1] == "--collect":
        collect(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
