#!/usr/bin/env python3
"""Config-5 single-frame latency probe: one 1280x960 pair, liveDisparity matcher
create(0, 256, 9, 8*81, 32*81), device-resident, per-call time and per-stage times
(mvsv_profile_*).  Env knobs of the library (MVSV_TRI_STATS, MVSV_STRIP_WAVES, ...)
apply.

    python tools/c5_frame.py [--frames 1] [--iters 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import numpy as np
    import torch
    import mvstereovision3_amd as mvsv

    W, H, D = 1280, 960, 256
    m = mvsv.StereoSGBM.create(0, D, 9, 8 * 81, 32 * 81)
    pairs = [mvsv.synth_pair(0x5EED0000 + i, W, H, 0, D) for i in range(a.frames)]
    dev = torch.device("cuda", 0)
    L = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
    R = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
    out = torch.empty((a.frames, H, W), dtype=torch.int16, device=dev)
    iters = 1 if (os.environ.get("MVSV_TRI_STATS") or os.environ.get("MVSV_TRI_TRACE")) else a.iters
    for _ in range(3 if iters > 1 else 1):
        m.compute(L, R, out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        m.compute(L, R, out)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1e3
    stages = {}
    if iters > 1:
        from mvstereovision3_amd import _lib
        ctx = _lib.context(0)
        _lib.profile_reset(ctx)
        _lib.profile_enable(ctx, True)
        for _ in range(10):
            m.compute(L, R, out)
        torch.cuda.synchronize()
        _lib.profile_enable(ctx, False)
        stages = {k: round(v[0] / 10, 4) for k, v in _lib.profile_read(ctx).items() if v[1]}
    print(json.dumps({"frames": a.frames, "ms_per_call": round(ms, 4),
                      "ms_per_frame": round(ms / a.frames, 4), "stages_ms": stages,
                      "env": {k: v for k, v in os.environ.items() if k.startswith("MVSV_")}}))


if __name__ == "__main__":
    main()
