#!/usr/bin/env python3
"""Per-config measurement table (BASELINE.md "What will be measured").

One JSON line per BASELINE config / variant, device-resident steady state
(inputs in HBM, K timed steps after W warm-up steps, median of per-step HIP
event times and the mean over the whole timed region), each with the roof it
is quoted against:

* SGBM 8 paths: HBM roof, §8(d) compulsory bytes 4*W*H*(1+D) per frame;
* SGBM 5 paths and BM: VALU roof (§8(d): ~50 and ~7 int16 ops per
  (pixel, disparity), MI355X packed-int16 VALU peak 157.3 T ops/s =
  2 x 78.6 T lane-ops/s);
* config 4 end-to-end: pinned host frames -> H2D -> compute -> D2H, 8 frames
  per step, copy and compute on one stream (the PCIe-inclusive rate);
* bm_match kernel: its HIP-event launch time next to the whole BM step.

Run on the GPU box: python tools/bench_configs.py [--steps K --warmup W] > table.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK = 8.0e12           # B/s
VALU_INT16_PEAK = 157.3e12  # packed int16 ops/s
OPS_PER_PXD = {"sgbm5": 50, "sgbm8": 82, "bm": 7}
SEED0 = 0x5EED0000
CFG = os.path.join(ROOT, "tests", "golden", "configs")


def timed(fn, steps, warmup):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(steps):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    per = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]
    return wall / steps * 1e3, statistics.median(per)


def sgbm_matcher(mvsv, mode):
    m = mvsv.StereoSGBM.create(0, 0, 0, 0, 0)
    assert mvsv.Disparity.loadSGBMParameters(os.path.join(CFG, "sgbm.yml"), m, mvsv.sgbmParameters())
    m.setMode(mode)
    return m


def frames(mvsv, n, W, H, minD, D, dev):
    import numpy as np
    import torch
    pairs = [mvsv.synth_pair(SEED0 + i, W, H, minD, D) for i in range(n)]
    L = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
    R = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
    return L, R


def line(name, W, H, D, n, mean_ms, med_ms, roof, extra=None):
    px = W * H * n
    rec = {"config": name, "width": W, "height": H, "num_disparities": D, "frames_per_step": n,
           "mean_ms_per_step": round(mean_ms, 4), "median_ms_per_step": round(med_ms, 4),
           "mpix_s": round(px / (med_ms / 1e3) / 1e6, 1)}
    kind, amount = roof
    t = med_ms / 1e3
    if kind == "hbm":
        rec["roof"] = {"bound": "hbm", "achieved_GBps": round(amount / t / 1e9, 1),
                       "frac": round(amount / t / HBM_PEAK, 4),
                       "bytes": "4*W*H*(1+D) per frame (SURVEY.md §8(d))"}
    else:
        rec["roof"] = {"bound": "valu", "achieved_Tops": round(amount / t / 1e12, 2),
                       "frac": round(amount / t / VALU_INT16_PEAK, 4),
                       "ops": f"{kind} int16 ops per (pixel, disparity) x W*H*D (SURVEY.md §8(d))"}
    rec.update(extra or {})
    print(json.dumps(rec), flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    import torch

    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd import _lib
    dev = torch.device("cuda", 0)
    K, Wm = args.steps, args.warmup

    # configs 1-2: StereoBM 640x480 (bm.yml; StereoBM(64, 9) OpenCV defaults)
    for name, make, D in (("config1_bm_yml_640x480", "yml", 80), ("config2_bm_d64_bs9_640x480", "d64", 64)):
        if make == "yml":
            b = mvsv.StereoBM.create(0, 21)
            assert mvsv.Disparity.loadBMParameters(os.path.join(CFG, "bm.yml"), b)
        else:
            b = mvsv.StereoBM.create(64, 9)
        for n in (1, 8):
            L, R = frames(mvsv, n, 640, 480, 0, D, dev)
            out = torch.empty((n, 480, 640), dtype=torch.int16, device=dev)
            ctx = _lib.context(0)
            _lib.profile_reset(ctx)
            _lib.profile_enable(ctx, True)
            mean, med = timed(lambda: b.compute(L, R, out), K, Wm)
            _lib.profile_enable(ctx, False)
            prof = _lib.profile_read(ctx)
            bm_ms, bm_n = prof.get("bm_match", (0.0, 0))
            line(name, 640, 480, D, n, mean, med, ("bm", OPS_PER_PXD["bm"] * 640 * 480 * D * n),
                 {"bm_match_kernel_ms_per_launch": round(bm_ms / max(bm_n, 1), 4)})
            # VALU roof uses the bm ops count; label it
    # config 3: SGBM sgbm.yml 640x480, 5 paths (mode 0) and 8 paths (mode 1)
    for mode in (0, 1):
        m = sgbm_matcher(mvsv, mode)
        for n in (1, 8):
            L, R = frames(mvsv, n, 640, 480, 1, 128, dev)
            out = torch.empty((n, 480, 640), dtype=torch.int16, device=dev)
            mean, med = timed(lambda: m.compute(L, R, out), K, Wm)
            roof = ("hbm", 4 * 640 * 480 * 129 * n) if mode == 1 else \
                ("sgbm5", OPS_PER_PXD["sgbm5"] * 640 * 480 * 128 * n)
            if roof[0] == "sgbm5":
                roof = ("sgbm5", roof[1])
            line(f"config3_sgbm_yml_640x480_{'8path' if mode else '5path'}", 640, 480, 128, n,
                 mean, med, roof, {"mode": "MODE_HH" if mode else "MODE_SGBM"})
    # config 4 per GPU: 1280x960, 8 frames, 8 paths -- device-resident and end-to-end
    m = sgbm_matcher(mvsv, 1)
    n, W, H = 8, 1280, 960
    L, R = frames(mvsv, n, W, H, 1, 128, dev)
    out = torch.empty((n, H, W), dtype=torch.int16, device=dev)
    mean, med = timed(lambda: m.compute(L, R, out), K, Wm)
    line("config4_sgbm_1280x960_8path_device_resident", W, H, 128, n, mean, med,
         ("hbm", 4 * W * H * 129 * n))
    hL = L.cpu().pin_memory()
    hR = R.cpu().pin_memory()
    hO = torch.empty((n, H, W), dtype=torch.int16).pin_memory()

    def e2e():
        L.copy_(hL, non_blocking=True)
        R.copy_(hR, non_blocking=True)
        m.compute(L, R, out)
        hO.copy_(out, non_blocking=True)

    mean, med = timed(e2e, K, Wm)
    line("config4_sgbm_1280x960_8path_end_to_end_pcie", W, H, 128, n, mean, med,
         ("hbm", 4 * W * H * 129 * n), {"note": "pinned H2D + compute + D2H on one stream"})
    # SGBM 5 paths at 1280x960 (VALU roof)
    m5 = sgbm_matcher(mvsv, 0)
    mean, med = timed(lambda: m5.compute(L, R, out), K, Wm)
    line("sgbm_1280x960_5path_device_resident", W, H, 128, n, mean, med,
         ("sgbm5", OPS_PER_PXD["sgbm5"] * W * H * 128 * n))
    # config 5 matcher (liveDisparity: create(0, 256, 9, 648, 2592), MODE_SGBM)
    # on one frame -- the live-camera latency -- and on the stream's batch of 8,
    # device-resident (tools/bench_stream.py measures the host-to-host stream)
    m256 = mvsv.StereoSGBM.create(0, 256, 9, 648, 2592)
    for n5 in (1, 8):
        L5, R5 = frames(mvsv, n5, W, H, 0, 256, dev)
        out5 = torch.empty((n5, H, W), dtype=torch.int16, device=dev)
        mean, med = timed(lambda: m256.compute(L5, R5, out5), K, Wm)
        line("config5_sgbm_1280x960_d256_device_resident", W, H, 256, n5, mean, med,
             ("sgbm5", OPS_PER_PXD["sgbm5"] * W * H * 256 * n5), {"mode": "MODE_SGBM"})
    mvsv.synchronize()


if __name__ == "__main__":
    main()
