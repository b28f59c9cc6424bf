#!/usr/bin/env python3
"""Per-call time of small repeated launches with and without HIP-graph replay
(MVSV_GRAPHS=0/1 are read per context: a fresh context per variant).

    python tools/graph_ab.py [--calls 200]
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
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    import numpy as np
    import torch
    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd import _lib
    dev = torch.device("cuda", 0)
    cfg = os.path.join(ROOT, "tests", "golden", "configs")
    res = {}
    for g in ("0", "1"):
        os.environ["MVSV_GRAPHS"] = g
        ctx = _lib.Context(0)
        with _lib.use_context(ctx):
            cases = []
            for mode in (0, 1):
                m = mvsv.StereoSGBM.create(0, 0, 0, 0, 0)
                assert mvsv.Disparity.loadSGBMParameters(os.path.join(cfg, "sgbm.yml"), m, mvsv.sgbmParameters())
                m.setMode(mode)
                cases.append((f"config3_mode{mode}_1frame", m, 640, 480, 1, 128))
            cases.append(("config2_bm_1frame", mvsv.StereoBM.create(64, 9), 640, 480, 0, 64))
            b1 = mvsv.StereoBM.create(0, 21)
            assert mvsv.Disparity.loadBMParameters(os.path.join(cfg, "bm.yml"), b1)
            cases.append(("config1_bm_1frame", b1, 640, 480, 0, 80))
            for name, m, W, H, minD, D in cases:
                Lh, Rh = mvsv.synth_pair(0x5EED0000, W, H, minD, D)
                L = torch.from_numpy(Lh).to(dev)
                R = torch.from_numpy(Rh).to(dev)
                out = torch.empty((H, W), dtype=torch.int16, device=dev)
                for _ in range(5):
                    m.compute(L, R, out)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.calls):
                    m.compute(L, R, out)
                torch.cuda.synchronize()
                res.setdefault(name, {})[f"graphs={g}"] = round((time.perf_counter() - t0) / a.calls * 1e3, 4)
        ctx.close()
    print(json.dumps({"ms_per_call": res}))


if __name__ == "__main__":
    main()
