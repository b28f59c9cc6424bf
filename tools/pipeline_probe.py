"""Probe: does splitting a frame batch over K contexts (own streams, own
buffers) overlap the latency-bound stages?  Prints ms per 8-frame batch for
K = 1, 2, 4 contexts and checks the outputs are identical.
Usage (on the GPU box): python tools/pipeline_probe.py [--steps 10]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--frames", type=int, default=8)
    a = ap.parse_args()
    import numpy as np
    import torch
    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd import _lib

    lib = _lib.lib()
    W, H, F = 1280, 960, a.frames
    m = mvsv.StereoSGBM.create(0, 0, 0, 0, 0)
    mvsv.Disparity.loadSGBMParameters(os.path.join(ROOT, "tests/golden/configs/sgbm.yml"), m,
                                      mvsv.sgbmParameters())
    m.setMode(1)
    pd = m.params()
    host = [mvsv.synth_pair(0x5EED0000 + i, W, H, pd["min_disparity"], pd["num_disparities"])
            for i in range(F)]
    dev = torch.device("cuda", 0)
    Lt = torch.from_numpy(np.stack([h[0] for h in host])).to(dev)
    Rt = torch.from_numpy(np.stack([h[1] for h in host])).to(dev)
    p = _lib.SgbmParams(**{k: pd[k] for k in _lib.SGBM_FIELDS})
    results = {}
    for K in (1, 2, 4):
        ctxs = []
        for _ in range(K):
            c = ctypes.c_void_p()
            assert lib.mvsv_create(ctypes.byref(c), 0) == 0
            assert lib.mvsv_use_own_stream(c) == 0
            ctxs.append(c)
        out = torch.empty((F, H, W), dtype=torch.int16, device=dev)
        per = F // K

        def step():
            for i, c in enumerate(ctxs):
                o = i * per * W * H
                rc = lib.mvsv_sgbm_device(c, per, Lt.data_ptr() + o, W, W * H, Rt.data_ptr() + o, W,
                                          W * H, W, H, ctypes.byref(p), out.data_ptr() + 2 * o, W,
                                          W * H)
                assert rc == 0, lib.mvsv_last_error(c)

        def sync():
            for c in ctxs:
                assert lib.mvsv_synchronize(c) == 0

        for _ in range(3):
            step()
        sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        sync()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        results[K] = out.clone()
        same = bool(torch.equal(results[K], results[1]))
        print(f"contexts={K} frames/ctx={per} ms_per_batch={ms:.3f} Mpix/s={F * W * H / ms / 1e3:.1f} "
              f"same_as_K1={same}", flush=True)
        for c in ctxs:
            lib.mvsv_destroy(c)


if __name__ == "__main__":
    main()
