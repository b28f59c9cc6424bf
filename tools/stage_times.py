"""Per-stage device times (HIP events, ms per call) of one SGBM configuration.

Usage (on the GPU box): python tools/stage_times.py [--frames F] [--width W --height H]
    [--ndisp D] [--mode 0|1] [--p1 P1 --p2 P2 --bs BS] [--steps K]
    [--speckle-window N --speckle-range R]
Defaults: config 5 (liveDisparity: create(0, 256, 9, 648, 2592), MODE_SGBM, one
1280x960 frame).  Env knobs (MVSV_PATH_SCHEDULE, MVSV_STRIP_WAVES, ...) apply."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=960)
    ap.add_argument("--ndisp", type=int, default=256)
    ap.add_argument("--mind", type=int, default=0)
    ap.add_argument("--bs", type=int, default=9)
    ap.add_argument("--p1", type=int, default=648)
    ap.add_argument("--p2", type=int, default=2592)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--speckle-window", type=int, default=0)
    ap.add_argument("--speckle-range", type=int, default=0)
    a = ap.parse_args()
    import numpy as np
    import torch
    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd import _lib
    m = mvsv.StereoSGBM.create(a.mind, a.ndisp, a.bs, a.p1, a.p2, 0, 0, 0, a.speckle_window, a.speckle_range)
    m.setMode(a.mode)
    host = [mvsv.synth_pair(0x5EED0000 + i, a.width, a.height, a.mind, a.ndisp) for i in range(a.frames)]
    L = torch.from_numpy(np.stack([h[0] for h in host])).cuda()
    R = torch.from_numpy(np.stack([h[1] for h in host])).cuda()
    out = torch.empty((a.frames, a.height, a.width), dtype=torch.int16, device="cuda")
    for _ in range(3):
        m.compute(L, R, out)
    torch.cuda.synchronize()
    ctx = _lib.context(0)
    _lib.profile_reset(ctx)
    _lib.profile_enable(ctx, True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        m.compute(L, R, out)
    e1.record()
    torch.cuda.synchronize()
    _lib.profile_enable(ctx, False)
    prof = _lib.profile_read(ctx)
    print(json.dumps({"frames": a.frames, "size": [a.width, a.height], "ndisp": a.ndisp, "mode": a.mode,
                      "ms_per_call": round(e0.elapsed_time(e1) / a.steps, 4),
                      "stages": {k: round(v[0] / a.steps, 4) for k, v in prof.items() if v[1]},
                      "env": {k: v for k, v in os.environ.items() if k.startswith("MVSV_")}}))


if __name__ == "__main__":
    main()
