"""Throughput with B batches in flight: B contexts (each its own HIP stream and
cached buffers) take consecutive steps of the bench workload round-robin, with
no host synchronisation between steps; compared with one context.

Usage (on the GPU box): python tools/concurrent_batches.py [--inflight 1 2 3] [--steps 24]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inflight", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--config5", action="store_true",
                    help="liveDisparity parameters: create(0, 256, 9, 648, 2592), MODE_SGBM")
    a = ap.parse_args()
    import numpy as np
    import torch
    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd import _lib
    W, H, F = 1280, 960, a.frames
    if a.config5:
        m = mvsv.StereoSGBM.create(0, 256, 9, 648, 2592)
    else:
        m = mvsv.StereoSGBM.create(0, 0, 0, 0, 0)
        mvsv.Disparity.loadSGBMParameters(os.path.join(ROOT, "tests/golden/configs/sgbm.yml"), m,
                                          mvsv.sgbmParameters())
        m.setMode(a.mode)
    pd = m.params()
    host = [mvsv.synth_pair(0x5EED0000 + i, W, H, pd["min_disparity"], pd["num_disparities"])
            for i in range(F)]
    dev = torch.device("cuda", 0)
    Lt = torch.from_numpy(np.stack([h[0] for h in host])).to(dev)
    Rt = torch.from_numpy(np.stack([h[1] for h in host])).to(dev)
    lib = _lib.lib()
    p = _lib.SgbmParams(**{k: pd[k] for k in _lib.SGBM_FIELDS})
    res = {}
    for nb in a.inflight:
        ctxs, outs = [], []
        for _ in range(nb):
            c = ctypes.c_void_p()
            assert lib.mvsv_create(ctypes.byref(c), 0) == 0
            ctxs.append(c)
            outs.append(torch.empty((F, H, W), dtype=torch.int16, device=dev))

        def step(i):
            c, o = ctxs[i % nb], outs[i % nb]
            rc = lib.mvsv_sgbm_device(c, F, Lt.data_ptr(), W, W * H, Rt.data_ptr(), W, W * H, W, H,
                                      ctypes.byref(p), o.data_ptr(), W, W * H)
            assert rc == 0, lib.mvsv_last_error(c)

        for i in range(2 * nb):
            step(i)
        for c in ctxs:
            assert lib.mvsv_synchronize(c) == 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i)
        for c in ctxs:
            assert lib.mvsv_synchronize(c) == 0
        t1 = time.perf_counter()
        ms = (t1 - t0) / a.steps * 1e3
        same = all(torch.equal(outs[0], o) for o in outs)
        res[nb] = {"ms_per_step": round(ms, 4), "mpix_s": round(F * W * H / ms / 1e3, 1), "outputs_equal": same}
        for c in ctxs:
            lib.mvsv_destroy(c)
        del outs
        torch.cuda.empty_cache()
    print(json.dumps({"inflight": res, "frames_per_step": F, "mode": a.mode}))


if __name__ == "__main__":
    main()
