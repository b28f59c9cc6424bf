"""In-process A/B of libmvsv.so variants on the bench workload.

Loads every variants/*.so (RTLD_LOCAL, one context each, same HIP runtime as
torch), runs the same device batch through each in round-robin for several
rounds and prints per-stage medians -- box-to-box and warm-up drift cancel out.
Usage (on the GPU box): python tools/ab_inproc.py [--rounds R] [--steps K] [variant.so ...]
"""
import argparse
import ctypes
import glob
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--mode", type=int, default=1)
    a = ap.parse_args()
    import numpy as np
    import torch
    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd import _lib

    libs = a.libs or sorted(glob.glob(os.path.join(ROOT, "variants", "*.so")))
    W, H, F = 1280, 960, 8
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
    outs = {}
    runs = []
    for path in libs:
        lib = _lib._declare(ctypes.CDLL(path, mode=os.RTLD_LOCAL), strict=False)
        ctx = ctypes.c_void_p()
        assert lib.mvsv_create(ctypes.byref(ctx), 0) == 0
        lib.mvsv_set_stream(ctx, None)
        p = _lib.SgbmParams(**{k: pd[k] for k in _lib.SGBM_FIELDS})
        out = torch.empty((F, H, W), dtype=torch.int16, device=dev)
        outs[path] = out
        runs.append((os.path.basename(path), lib, ctx, p, out))

    def step(lib, ctx, p, out):
        rc = lib.mvsv_sgbm_device(ctx, F, Lt.data_ptr(), W, W * H, Rt.data_ptr(), W, W * H, W, H,
                                  ctypes.byref(p), out.data_ptr(), W, W * H)
        assert rc == 0, lib.mvsv_last_error(ctx)

    res = {r[0]: {"total": []} for r in runs}
    for name, lib, ctx, p, out in runs:  # warm-up
        step(lib, ctx, p, out)
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, lib, ctx, p, out in runs:
            lib.mvsv_profile_reset(ctx)
            lib.mvsv_profile_enable(ctx, 1)
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(a.steps):
                step(lib, ctx, p, out)
            s1.record()
            torch.cuda.synchronize()
            lib.mvsv_profile_enable(ctx, 0)
            ms = (ctypes.c_double * _lib.NUM_STAGES)()
            cnt = (ctypes.c_int * _lib.NUM_STAGES)()
            lib.mvsv_profile_read(ctx, ms, cnt, _lib.NUM_STAGES)
            res[name]["total"].append(s0.elapsed_time(s1) / a.steps)
            for i in range(_lib.NUM_STAGES):
                n = lib.mvsv_profile_stage_name(i).decode() or f"stage{i}"
                if cnt[i]:
                    res[name].setdefault(n, []).append(ms[i] / a.steps)
    base = outs[libs[0]]
    for name, lib, ctx, p, out in runs:
        same = bool(torch.equal(out, base))
        med = {k: round(statistics.median(v), 4) for k, v in res[name].items()}
        print(f"{name:24s} same_as_first={same} {med}")


if __name__ == "__main__":
    main()
