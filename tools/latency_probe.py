"""Per-stage latency of small SGBM launches (the live-camera shapes):
config 3 (640x480, configs/sgbm.yml, 8 paths) and config 5 (1280x960,
create(0, 256, 9, 648, 2592), MODE_SGBM) at 1 and 2 frames, device-resident,
HIP-event stage times from the library's profiler.
Usage (GPU box): python tools/latency_probe.py"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mvstereovision3_amd as mvsv  # noqa: E402
from mvstereovision3_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)


def run(name, m, W, H, D, n, steps=30):
    pairs = [mvsv.synth_pair(0x5EED0000 + i, W, H, 0, D) for i in range(n)]
    L = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
    R = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
    out = torch.empty((n, H, W), dtype=torch.int16, device=dev)
    for _ in range(5):
        m.compute(L, R, out)
    torch.cuda.synchronize()
    ctx = _lib.context(0)
    _lib.profile_reset(ctx)
    _lib.profile_enable(ctx, True)
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        m.compute(L, R, out)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    _lib.profile_enable(ctx, False)
    prof = _lib.profile_read(ctx)
    st = {k: round(v[0] / steps, 4) for k, v in prof.items() if v[1]}
    print(f"{name} frames={n}: median {statistics.median(ts) * 1e3:.3f} ms host-timed; stages {st}", flush=True)


cfg3 = mvsv.StereoSGBM.create(1, 128, 13, 0, 0, 0, 0, 0, 150, 2, 1)
cfg5 = mvsv.StereoSGBM.create(0, 256, 9, 648, 2592)
for n in (1, 2, 8):
    run("config3_640x480_8path", cfg3, 640, 480, 128, n)
    run("config5_1280x960_d256", cfg5, 1280, 960, 256, n)
