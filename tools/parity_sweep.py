"""Randomized parity sweep (GPU box): many random StereoSGBM / StereoBM cases --
shapes, parameters, OpenCV variants, frame batches and every launch-shape option
(SGBM path schedule, strip width, strip order; BM tile rows, general kernel) -- computed on the
GPU through the package and checked bit-exactly against the C oracle (test
infrastructure; the oracle frames run on a process pool of host threads).

Usage (GPU box):  python tools/parity_sweep.py [--sgbm 200] [--bm 200] [--seed 1]
Prints one line per mismatch and a summary; exit status 1 on any mismatch.
"""
import argparse
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def rand_pair(rng, H, W, shift, kind):
    if kind == 0:
        from scipy.ndimage import uniform_filter
        L = uniform_filter(rng.integers(0, 256, (H, W)).astype(float), 3).round().astype(np.uint8)
    elif kind == 1:
        L = (rng.integers(0, 4, (H, W)) * 60).astype(np.uint8)
        L[:, W // 3:W // 2] = 128
    else:
        L = rng.integers(0, 256, (H, W)).astype(np.uint8)
    R = np.roll(L, -shift, axis=1)
    R = np.clip(R.astype(int) + rng.integers(-2, 3, R.shape), 0, 255).astype(np.uint8)
    return L, R


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sgbm", type=int, default=200)
    ap.add_argument("--bm", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--large", type=int, default=0,
                    help="extra SGBM cases at 640x480 / 1280x960 with 4-8 frame batches")
    ap.add_argument("--bits", type=int, default=0,
                    help="SGBM cases in the bit-sliced regime (MODE_HH, D 128, P1 2 / P2 5, "
                         "uniquenessRatio 0): random shapes, batches, schedules, bit-sliced on / off")
    ap.add_argument("--bits-large", type=int, default=0,
                    help="bit-sliced-regime cases at 640x480 / 1280x960, 1-8 frames")
    a = ap.parse_args()
    import torch

    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd import _lib
    from oracle import pyoracle
    pyoracle.lib()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(a.seed)
    pool = ThreadPoolExecutor(16)
    bad = 0
    jobs = []

    for i in range(a.sgbm):
        n = int(rng.choice([1, 1, 2, 3]))
        H, W = int(rng.integers(16, 200)), int(rng.integers(64, 360))
        D = int(rng.choice([16, 32, 48, 64, 96, 128, 256]))
        minD = int(rng.integers(-8, 8))
        while W + min(minD, 0) - max(minD + D, 0) < 16 and D > 16:
            D = max(16, (D // 2) // 16 * 16)
        if W + min(minD, 0) - max(minD + D, 0) < 16:
            continue
        bs = int(rng.choice([0, 1, 3, 5, 7, 9, 11, 13, 15, 17]))
        P1 = int(rng.choice([0, 2, 8, 72, 300]))
        P2 = int(rng.choice([0, 5, 15, 40, 288, 2000, 4000]))
        kw = dict(minDisparity=minD, numDisparities=D, blockSize=bs, P1=P1, P2=P2,
                  disp12MaxDiff=int(rng.integers(-1, 4)), preFilterCap=int(rng.choice([0, 15, 31, 63])),
                  uniquenessRatio=int(rng.choice([-1, 0, 5, 15])),
                  speckleWindowSize=int(rng.choice([0, 0, 10, 50])), speckleRange=int(rng.choice([1, 2, 4])),
                  mode=int(rng.integers(0, 2)))
        variant = int(rng.integers(0, 4))
        sched = int(rng.choice([0, 0, 1, 2]))
        waves = int(rng.choice([0, 0, 4, 7, 8, 15]))
        pairs = [rand_pair(rng, H, W, int(rng.integers(0, min(D, 64))), int(rng.integers(0, 3)))
                 for _ in range(n)]
        m = mvsv.StereoSGBM.create(**kw)
        m.setVariant(variant)
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, sched)
        _lib.set_option(_lib.OPT_STRIP_WAVES, waves)
        _lib.set_option(_lib.OPT_STRIP_TICKETS, int(rng.integers(0, 2)))
        res = int(rng.choice([1, 1, 1, 0]))  # cost residual plane where exact (round 4) / forced off
        _lib.set_option(_lib.OPT_COST_RESIDUAL, res)
        try:
            if n == 1:
                got = m.compute(*pairs[0])[None]
            else:
                Lb = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
                Rb = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
                out = torch.empty((n, H, W), dtype=torch.int16, device=dev)
                m.compute(Lb, Rb, out)
                got = out.cpu().numpy()
        except mvsv.MvsvError as ex:
            print(f"GPU ERROR sgbm #{i} {H}x{W} {kw}: {ex}", flush=True)
            bad += 1
            continue
        p = {k: v for k, v in m.params().items() if k != "variant"}
        for j, (L, R) in enumerate(pairs):
            tag = f"sgbm #{i} frame {j}/{n} {H}x{W} {kw} variant={variant} sched={sched} waves={waves} res={res}"
            jobs.append((tag, got[j], pool.submit(pyoracle.sgbm, L, R, p, variant)))
    _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    _lib.set_option(_lib.OPT_STRIP_WAVES, 0)

    for i in range(a.large):  # batch shapes: wide strips, lines after the strips
        W, H = (640, 480) if rng.integers(0, 3) else (1280, 960)
        n = int(rng.choice([1, 4, 8])) if W == 640 else int(rng.choice([1, 2, 4]))
        D = int(rng.choice([16, 64, 128, 256]))  # round 6: D 16 (captureDisparity), one-frame launches
        kw = dict(minDisparity=int(rng.integers(-4, 4)), numDisparities=D,
                  blockSize=int(rng.choice([3, 5, 9, 13])), P1=int(rng.choice([0, 2, 8, 648])),
                  P2=int(rng.choice([0, 5, 32, 2592])), disp12MaxDiff=int(rng.integers(-1, 3)),
                  preFilterCap=int(rng.choice([0, 31, 63])), uniquenessRatio=int(rng.choice([0, 10])),
                  speckleWindowSize=int(rng.choice([0, 150])), speckleRange=2, mode=int(rng.integers(0, 2)))
        m = mvsv.StereoSGBM.create(**kw)
        tickets = int(rng.integers(0, 2))  # strip order of launches larger than the CU count
        _lib.set_option(_lib.OPT_STRIP_TICKETS, tickets)
        kw["strip_tickets"] = tickets
        res = int(rng.choice([1, 1, 1, 0]))
        _lib.set_option(_lib.OPT_COST_RESIDUAL, res)
        kw["cost_residual"] = res
        pairs = [mvsv.synth_pair(int(rng.integers(0, 1 << 30)), W, H, max(kw["minDisparity"], 0), D)
                 for _ in range(n)]
        Lb = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
        Rb = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
        out = torch.empty((n, H, W), dtype=torch.int16, device=dev)
        m.compute(Lb, Rb, out)
        got = out.cpu().numpy()
        p = {k: v for k, v in m.params().items() if k != "variant"}
        for j, (L, R) in enumerate(pairs):
            jobs.append((f"large #{i} frame {j}/{n} {W}x{H} {kw}", got[j], pool.submit(pyoracle.sgbm, L, R, p)))
    _lib.set_option(_lib.OPT_STRIP_TICKETS, 1)
    _lib.set_option(_lib.OPT_COST_RESIDUAL, 1)

    # the bit-sliced pipeline (round 5 MODE_HH, round 6 MODE_SGBM): strips +
    # fused R->L / WTA for batches, the side-by-side chains for small launches,
    # forced off
    for i in range(a.bits + a.bits_large):
        large = i >= a.bits
        if large:
            W, H = (640, 480) if rng.integers(0, 2) else (1280, 960)
            n = int(rng.choice([1, 2, 4, 8])) if W == 640 else int(rng.choice([1, 2, 3]))
        else:
            n = int(rng.choice([1, 1, 2, 3, 5]))
            H, W = int(rng.integers(8, 160)), int(rng.integers(150, 420))
        minD = int(rng.integers(-8, 8))
        if W + min(minD, 0) - max(minD + 128, 0) < 1:
            continue
        kw = dict(minDisparity=minD, numDisparities=128, blockSize=int(rng.choice([0, 1, 3, 5, 9, 13, 15])),
                  P1=int(rng.choice([0, 2])), P2=int(rng.choice([0, 5])), disp12MaxDiff=int(rng.integers(-1, 4)),
                  preFilterCap=int(rng.choice([0, 15, 31, 63])), uniquenessRatio=0,
                  speckleWindowSize=int(rng.choice([0, 0, 20, 150])), speckleRange=int(rng.choice([1, 2, 4])),
                  mode=int(rng.integers(0, 2)))  # round 6: MODE_SGBM is bit-sliced too
        variant = int(rng.integers(0, 4))
        sched = int(rng.choice([0, 0, 1, 2]))
        bits = int(rng.choice([1, 1, 1, 0]))
        m = mvsv.StereoSGBM.create(**kw)
        m.setVariant(variant)
        _lib.set_option(_lib.OPT_PATH_SCHEDULE, sched)
        _lib.set_option(_lib.OPT_BITSLICE, bits)
        if large:
            pairs = [mvsv.synth_pair(int(rng.integers(0, 1 << 30)), W, H, max(minD, 0), 128) for _ in range(n)]
        else:
            pairs = [rand_pair(rng, H, W, int(rng.integers(0, 64)), int(rng.integers(0, 3))) for _ in range(n)]
        try:
            Lb = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
            Rb = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
            out = torch.empty((n, H, W), dtype=torch.int16, device=dev)
            m.compute(Lb, Rb, out)
            got = out.cpu().numpy()
        except mvsv.MvsvError as ex:
            print(f"GPU ERROR bits #{i} {H}x{W} {kw}: {ex}", flush=True)
            bad += 1
            continue
        p = {k: v for k, v in m.params().items() if k != "variant"}
        for j, (L, R) in enumerate(pairs):
            tag = f"bits #{i} frame {j}/{n} {H}x{W} {kw} variant={variant} sched={sched} bitslice={bits}"
            jobs.append((tag, got[j], pool.submit(pyoracle.sgbm, L, R, p, variant)))
    _lib.set_option(_lib.OPT_PATH_SCHEDULE, 0)
    _lib.set_option(_lib.OPT_BITSLICE, 1)

    for i in range(a.bm):
        H, W = int(rng.integers(24, 200)), int(rng.integers(80, 400))
        D = int(rng.choice([16, 32, 48, 64, 80, 96, 112, 128, 144, 160]))
        bs = int(rng.choice([5, 7, 9, 11, 13, 15, 17, 19, 21, 23, 25]))
        minD = int(rng.integers(-8, 8))
        if bs >= min(H, W) or W - D - abs(minD) - bs < 8:
            continue
        p = dict(pre_filter_type=int(rng.integers(0, 2)), pre_filter_size=int(rng.choice([5, 9, 15])),
                 pre_filter_cap=int(rng.integers(1, 64)), block_size=bs, min_disparity=minD,
                 num_disparities=D, texture_threshold=int(rng.choice([0, 10, 100])),
                 uniqueness_ratio=int(rng.choice([0, 5, 15, 60])),
                 speckle_window_size=int(rng.choice([0, 0, 20])), speckle_range=int(rng.choice([0, 4, 32])),
                 disp12_max_diff=int(rng.choice([-1, 0, 1, 3])))
        ty = int(rng.choice([0, 0, 1, 8, 24, 64]))
        L, R = rand_pair(rng, H, W, int(rng.integers(0, min(D, 48))), int(rng.integers(0, 3)))
        m = mvsv.StereoBM.create(D, bs)
        for k, v in p.items():
            if k not in ("block_size", "num_disparities"):
                setattr(m._params, k, v)
        _lib.set_option(_lib.OPT_BM_TILE_ROWS, ty)
        try:
            got = m.compute(L, R)
        except mvsv.MvsvError as ex:
            if ty > 0 and "LDS" in str(ex):
                continue  # a forced tile height whose LDS image does not fit
            print(f"GPU ERROR bm #{i} {H}x{W} {p} ty={ty}: {ex}", flush=True)
            bad += 1
            continue
        tag = f"bm #{i} {H}x{W} {p} ty={ty}"
        jobs.append((tag, got, pool.submit(pyoracle.bm, L, R, p)))
    _lib.set_option(_lib.OPT_BM_TILE_ROWS, 0)
    mvsv.synchronize()

    for done, (tag, got, fut) in enumerate(jobs):
        if done % 50 == 0:
            print(f"checked {done} / {len(jobs)}", flush=True)  # progress (a quiet run looks hung)
        try:
            want = fut.result()
        except ValueError as ex:
            print(f"ORACLE ERROR {tag}: {ex}", flush=True)
            bad += 1
            continue
        if not np.array_equal(got, want):
            bad += 1
            idx = np.argwhere(got != want)
            print(f"MISMATCH {tag}: {len(idx)} px, first {[(int(y), int(x), int(got[y, x]), int(want[y, x])) for y, x in idx[:4]]}",
                  flush=True)
    print(f"parity sweep: {len(jobs)} frames, {bad} mismatching", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
