#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X stereo disparity engine.

Metric (BASELINE.json): "Mpix disparities/sec (SGBM 128-disp, 8-path) at
1/2/4/8 GPUs; % HBM roofline".  Workload = BASELINE config 4, the largest
single-GPU configuration of the metric: StereoSGBM on 1280x960 synthetic
rectified pairs, configs/sgbm.yml values (minDisparity 1, 128 disparities,
blockSize 13, P1/P2 = OpenCV defaults 2/5, speckle 150/2) with mode forced to
MODE_HH (8 paths), a batch of 8 frames per GPU (config 4 = 64 frames over 8
GPUs; weak scaling: per-GPU work fixed).

One step = one batch of frames through the full StereoSGBM::compute path
(prefilter, cost volume, 8 path aggregations, WTA/uniqueness/sub-pixel/LR,
median, speckle) with inputs already resident in HBM, plus -- for N > 1 -- the
RCCL gather of the int16 maps to rank 0 (the only exchange step of the
frame-parallel batch mode).

Batches in flight (--inflight, default 2): consecutive steps run on separate HIP
streams, each with its own context (cached volumes) and output, so the kernels of
one batch overlap those of the next (e.g. the latency-bound final kernel of step
k beside the cost kernel of step k+1) -- the serving shape of the batch mode;
every step still computes its whole batch.  value = frames of all K steps / wall
time.  --inflight 1 runs the steps strictly one after the other
(single_batch_ms reports that latency in every run).  The roofline's stage
times come from a separate one-in-flight pass (overlapped launches have no
kernel duration); profile rocprofv3 runs with --inflight 1 so its kernel
averages agree.

Run: python bench.py [--gpus N --steps K --warmup W].  With N > 1 and no
WORLD_SIZE in the environment, bench.py starts the N ranks itself (a child
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1`,
before any GPU call) and exits with its status; under an external launcher it
checks that WORLD_SIZE == N.  --dry rehearses the launcher and the gather on
CPU (gloo, a trivial host compute, no GPU and no oracle).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import socket
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SEED0 = 0x5EED0000
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SGBM_YML = os.path.join(ROOT, "tests", "golden", "configs", "sgbm.yml")
PROFILE_DIR = os.path.join(ROOT, "profiles", "r06")
PMC_FILE = os.path.join(PROFILE_DIR, "pmc_traffic.json")  # tools/pmc_traffic.py
SQ_FILE = os.path.join(PROFILE_DIR, "sq_summary.json")    # tools/sq_summary.py
KERNEL_SOURCES = os.path.join(ROOT, "mvstereovision3_amd", "csrc")
CPU_SHARE = 16  # host cores of one GPU's share on the GPU box

# MFMA is unused (integer min/add work, no dense contraction): a kernel is
# bound by HBM or by VALU issue; roofline.bound names the larger of the two
# MEASURED utilisations (PMC traffic / peak, SQ VALU busy cycles / SIMD cycles)
# of the dominant kernel, from summaries of the same kernel sources.


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=8, help="frames per GPU per step")
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=960)
    ap.add_argument("--mode", type=int, default=1, help="1 = MODE_HH (8 paths), 0 = 5 paths")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = the GPU's host-core share, <= 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--inflight", type=int, default=2,
                    help="batches in flight: consecutive steps on separate HIP streams / contexts "
                         "(their kernels overlap); 1 = strictly one step after the other")
    ap.add_argument("--profile-steps", type=int, default=200,
                    help="steps of the separate one-in-flight pass that times the stages (roofline)")
    ap.add_argument("--force-gather", action="store_true",
                    help="run the multi-rank path even for --gpus 1: torch.distributed.run "
                         "child, NCCL (RCCL) process group, dist.gather of the maps every step")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the per-config table (BASELINE configs 1, 2, 3, 5; single GPU only)")
    ap.add_argument("--dry", action="store_true",
                    help="CPU rehearsal of launcher + gather (gloo, trivial compute)")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """Start args.gpus ranks of this script under torch.distributed.run (a child
    process; nothing here has touched the GPU) and return its exit status."""
    if not args.dry:
        import torch
        have = torch.cuda.device_count()  # does not initialise the GPU on this image
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {have} GPUs visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def stage_bytes(stage, F, W, H, W1, D, ndir, acc, strips=True, res=False, bits=False, side=False):
    """Implementation HBM bytes of one step per stage ("Kernels").

    acc = bytes per (pixel, disparity) of a path-delta accumulator plane (0.5 for
    the 4-bit planes of the strip schedule when 3 * P2 <= 15, 1 when
    ndir * P2 <= 255, else 2).  strips = the sheared-strip schedule (D in
    {32, 64, 128, 256}): the strip kernel runs npass passes (down, + up for 8
    paths) that each read their cost input and write their own plane, the L->R
    line kernel reads its cost input and writes a plane, the final kernel reads C
    and every plane.  res = the direction passes read the nibble cost residual
    plane (0.5 B per cost, written by the cost kernel beside C) instead of C.
    bits = the bit-sliced MODE_HH pipeline (mvsv_bsgm.hip): the
    cost kernel writes C (read back only at best -+ 1) and the 4-bit C' planes,
    the strip passes read C' and write a 4-bit plane each, the L->R lines read
    C' and write a 3-bit plane, the R->L lines fused with the WTA read C', the
    three planes and the gathered costs.  bits + side = the bit-sliced
    small-launch form: every direction on its own chains writing a grouped 3-bit
    delta plane (48 B per padded pixel), the WTA reading C' and all of them.
    (Which form runs is what the library reports, mvsv_sgbm_plan.)
    """
    cells = W1 * H * D
    px = W * H
    npass = 2 if ndir == 8 else 1
    cin = 0.5 if res else 2
    if bits and side:
        W1q = (W1 + 3) // 4 * 4
        dirs_b = F * ndir * (W1q * H * 64 + W1q * H * 48)  # each chain reads C', writes its plane
        return {
            "prefilter": F * (2 * px + 2 * 8 * px),
            "cost_volume": F * (2 * 8 * px + 2.5 * cells + 2 * W1 * H),
            "path_aggregation": dirs_b,
            "final_wta_lr": F * (W1q * H * (64 + ndir * 48) + W1 * H * (2 + 8) + 6 * px),
            "post_filters": F * 4 * px,
        }.get(stage, 0)
    if bits:
        npb = 2 if ndir == 8 else 1  # strip passes (MODE_SGBM: down only)
        strip_b = F * cells * npb * (0.5 + 0.5)
        lines_b = F * cells * (0.5 + 0.375)  # L->R only: R->L runs with the WTA
        return {
            "prefilter": F * (2 * px + 2 * 8 * px),
            "cost_volume": F * (2 * 8 * px + 2.5 * cells + 2 * W1 * H),
            "path_aggregation": strip_b + lines_b,
            "path_strips": strip_b,
            "path_lines": lines_b,
            # R->L + WTA: C', two strip planes, the L->R plane, a 4-byte record
            # per pixel written and read back; the finish: minimum, gathered
            # costs, raw map and right-view keys per pixel
            "final_wta_lr": F * (cells * (0.5 + npb * 0.5 + 0.375) + W1 * H * (8 + 2 + 8) + 6 * px),
            "post_filters": F * 4 * px,
        }.get(stage, 0)
    if strips:
        planes = npass + 1
        strip_b = F * cells * npass * (cin + acc)
        lines_b = F * cells * (cin + acc)
        path_b = strip_b + lines_b
        final_b = F * (cells * (2 + planes * acc) + 2 * px)
    else:
        strip_b = lines_b = 0
        path_b = F * cells * ((2 + acc) + (ndir - 2) * (2 + 2 * acc))
        final_b = F * (cells * (2 + acc) + 2 * px)
    return {
        "prefilter": F * (2 * px + 2 * 8 * px),
        "cost_volume": F * (2 * 8 * px + (2 + (0.5 if res else 0)) * cells),
        "cost_fixup": 0,
        "path_aggregation": path_b,
        "path_strips": strip_b,
        "path_lines": lines_b,
        "final_wta_lr": final_b,
        "post_filters": F * 4 * px,
    }.get(stage, 0)


def _summary(path, workload, sha, what):
    """A committed counter summary, only if it is of this workload and these
    kernel sources: (dict or None, provenance note)."""
    if not os.path.exists(path):
        return None, f"no {what} summary ({os.path.relpath(path, ROOT)} absent)"
    try:
        js = json.load(open(path))
    except (OSError, ValueError):
        return None, f"{what} summary unreadable"
    if js.get("workload") != workload:
        return None, f"{what} summary is for another workload"
    if js.get("kernel_source_sha") != sha:
        return None, f"{what} summary is stale (kernel sources changed since)"
    return js, f"{os.path.relpath(path, ROOT)}, kernel sources {sha}"


def kernel_source_sha() -> str:
    h = hashlib.sha256()
    # the kernels and the host code that picks them (dispatch defaults, eligibility
    # gates, launch shapes) and the ABI header: a summary goes stale when any changes
    for p in sorted(glob.glob(os.path.join(KERNEL_SOURCES, "*.hip")) +
                    glob.glob(os.path.join(KERNEL_SOURCES, "*.hpp")) +
                    glob.glob(os.path.join(KERNEL_SOURCES, "*.cpp")) +
                    [os.path.join(ROOT, "include", "mvsv.h")]):
        h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


VALU_INT16_PEAK_TOPS = 157.3  # packed int16 ops/s x 1e-12 (2 x 78.6 T lane-ops/s)
OPS_PER_PXD = {"sgbm5": 50, "bm": 7}  # SURVEY.md §8(d) int16 ops per (pixel, disparity)


def config_table(mvsv, _lib, dev, steps=10, warmup=3):
    """The other BASELINE configs on this GPU: device-resident
    HIP-event median of `steps` steps after `warmup`, each with the roof SURVEY.md
    §8(d) quotes it against (HBM on 4*W*H*(1+D) bytes for 8 paths, VALU on its
    int16 op count for 5 paths and StereoBM) and a parity flag -- frame 0 of the
    output against the oracle, computed after all timing (oracles in threads)."""
    import numpy as np
    import torch
    from oracle import pyoracle

    cfg = os.path.join(ROOT, "tests", "golden", "configs")

    def timed(fn):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize(dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        ev[0].record()
        for i in range(steps):
            fn()
            ev[i + 1].record()
        torch.cuda.synchronize(dev)
        return statistics.median(ev[i].elapsed_time(ev[i + 1]) for i in range(steps))

    def frames(n, W, H, minD, D):
        pairs = [mvsv.synth_pair(SEED0 + i, W, H, minD, D) for i in range(n)]
        L = torch.from_numpy(np.stack([q[0] for q in pairs])).to(dev)
        R = torch.from_numpy(np.stack([q[1] for q in pairs])).to(dev)
        return pairs, L, R

    recs, checks = {}, []

    def add(name, W, H, D, n, ms, roof, pair, out0, oracle_fn, extra=None):
        t = ms / 1e3
        rec = {"width": W, "height": H, "num_disparities": D, "frames": n, "median_ms": round(ms, 4),
               "mpix_s": round(W * H * n / t / 1e6, 1)}
        kind, amount = roof
        if kind == "hbm":
            rec["roof"] = {"bound": "hbm", "achieved_GBps": round(amount / t / 1e9, 1),
                           "frac": round(amount / t / (HBM_PEAK_GBPS * 1e9), 4),
                           "model": "4*W*H*(1+D) bytes per frame"}
        else:
            rec["roof"] = {"bound": "valu", "achieved_Tops": round(amount / t / 1e12, 2),
                           "frac": round(amount / t / (VALU_INT16_PEAK_TOPS * 1e12), 4),
                           "model": f"{OPS_PER_PXD[kind]} int16 ops per (pixel, disparity)"}
        rec.update(extra or {})
        recs[name] = rec
        checks.append((name, pair, out0, oracle_fn))

    # configs 1-2: StereoBM 640x480 (configs/bm.yml; StereoBM(64, 9) OpenCV defaults)
    for name, D in (("config1_bm_yml_640x480", 80), ("config2_bm_d64_bs9_640x480", 64)):
        if D == 80:
            b = mvsv.StereoBM.create(0, 21)
            assert mvsv.Disparity.loadBMParameters(os.path.join(cfg, "bm.yml"), b)
        else:
            b = mvsv.StereoBM.create(64, 9)
        bp = b.params()
        for n in ((8,) if D == 80 else (1, 8)):
            pairs, L, R = frames(n, 640, 480, 0, D)
            out = torch.empty((n, 480, 640), dtype=torch.int16, device=dev)
            ctx = _lib.context(dev.index or 0)
            _lib.profile_reset(ctx)
            _lib.profile_enable(ctx, True)
            ms = timed(lambda: b.compute(L, R, out))
            _lib.profile_enable(ctx, False)
            bm_ms, bm_n = _lib.profile_read(ctx).get("bm_match", (0.0, 0))
            add(f"{name}_batch{n}", 640, 480, D, n, ms, ("bm", OPS_PER_PXD["bm"] * 640 * 480 * D * n),
                pairs[0], out[0].cpu().numpy(), lambda L0, R0, bp=bp: pyoracle.bm(L0, R0, bp),
                {"bm_match_kernel_ms": round(bm_ms / max(bm_n, 1), 4)})
    # config 3: SGBM configs/sgbm.yml 640x480, one frame (the live-camera case) and
    # a batch of 8, 5 paths (mode 0: what sgbm.yml selects) and 8 paths; and the
    # 5-path mode at the headline's 1280x960 batch of 8
    for mode in (0, 1):
        m = mvsv.StereoSGBM.create(0, 0, 0, 0, 0)
        assert mvsv.Disparity.loadSGBMParameters(os.path.join(cfg, "sgbm.yml"), m, mvsv.sgbmParameters())
        m.setMode(mode)
        p = {k: v for k, v in m.params().items() if k != "variant"}
        shapes = [(640, 480, 1), (640, 480, 8)] + ([(1280, 960, 8)] if mode == 0 else [])
        for W, H, n in shapes:
            pairs, L, R = frames(n, W, H, 1, 128)
            out = torch.empty((n, H, W), dtype=torch.int16, device=dev)
            ms = timed(lambda: m.compute(L, R, out))
            roof = ("hbm", 4 * W * H * 129 * n) if mode else ("sgbm5", OPS_PER_PXD["sgbm5"] * W * H * 128 * n)
            name = (f"config3_sgbm_yml_640x480_{'8path' if mode else '5path'}_batch{n}" if W == 640
                    else f"sgbm_{W}x{H}_d128_5path_batch{n}")
            add(name, W, H, 128, n, ms, roof, pairs[0], out[0].cpu().numpy(),
                lambda L0, R0, p=p: pyoracle.sgbm(L0, R0, p), {"mode": "MODE_HH" if mode else "MODE_SGBM"})
    # config 5: liveDisparity's create(0, 256, 9, 648, 2592) (trgt/liveDisparity.cpp:61,
    # MODE_SGBM, no speckle) at 1280x960: one frame and the stream's batch of 8
    m256 = mvsv.StereoSGBM.create(0, 256, 9, 648, 2592)
    p256 = {k: v for k, v in m256.params().items() if k != "variant"}
    for n in (1, 8):
        pairs, L, R = frames(n, 1280, 960, 0, 256)
        out = torch.empty((n, 960, 1280), dtype=torch.int16, device=dev)
        ms = timed(lambda: m256.compute(L, R, out))
        add(f"config5_sgbm_1280x960_d256_batch{n}", 1280, 960, 256, n, ms,
            ("sgbm5", OPS_PER_PXD["sgbm5"] * 1280 * 960 * 256 * n), pairs[0], out[0].cpu().numpy(),
            (lambda L0, R0, p=p256: pyoracle.sgbm(L0, R0, p)) if n == 1 else None, {"mode": "MODE_SGBM"})
    # the reference's other call sites: liveDisparity's
    # default create(0, 64, 9, 648, 2592) (trgt/liveDisparity.cpp:19-20,61) at
    # 1280x960 and captureDisparity's create(0, 16, 5, 200, 800)
    # (trgt/captureDisparity.cpp:24-25,196) at 640x480, one frame and a batch of 8
    for name, (mn, nd, bsz, p1, p2), (W, H) in (
            ("live_default_sgbm_d64_bs9", (0, 64, 9, 648, 2592), (1280, 960)),
            ("capture_sgbm_d16_bs5", (0, 16, 5, 200, 800), (640, 480))):
        mc = mvsv.StereoSGBM.create(mn, nd, bsz, p1, p2)
        pc = {k: v for k, v in mc.params().items() if k != "variant"}
        for n in (1, 8):
            pairs, L, R = frames(n, W, H, mn, nd)
            out = torch.empty((n, H, W), dtype=torch.int16, device=dev)
            ms = timed(lambda: mc.compute(L, R, out))
            add(f"{name}_{W}x{H}_batch{n}", W, H, nd, n, ms, ("sgbm5", OPS_PER_PXD["sgbm5"] * W * H * nd * n),
                pairs[0], out[0].cpu().numpy(),
                (lambda L0, R0, p=pc: pyoracle.sgbm(L0, R0, p)) if n == 1 else None, {"mode": "MODE_SGBM"})
    # config 5 as BASELINE states it: the sustained stream (host frames in, maps and
    # the 81 MeanDisparityDetection means out, the detection post-pass on every
    # frame; trgt/liveDisparity.cpp:61,82-101, src/MeanDisparityDetection.cpp:159-266)
    from tools.bench_stream import stream_measure
    sm = stream_measure(mvsv, frames=240, depth=24, batch=8, inflight=2, device_steps=5)
    recs["config5_stream_1280x960_d256_fps"] = {
        "width": 1280, "height": 960, "num_disparities": 256, "stream_fps": sm["stream_fps"],
        "stream_ms_per_frame": sm["stream_ms_per_frame"], "frames": sm["frames"], "depth": sm["depth"],
        "batch": sm["batch"], "inflight": sm["inflight"], "host_ms_per_frame": sm["host_ms_per_frame"],
        "device_resident_ms_per_frame_with_mean_grid": sm["device_resident_ms_per_frame"],
        "obstacle_tiles_found": sm["obstacle_tiles_found"],
        "note": "DisparityStream: host frames in, int16 map + 81 tile means out (PCIe incl.), "
                "MeanDisparityDetection build(MEAN_VALUE) + detectObstacles per frame, in the timing"}
    # parity: frame 0 of every config against the oracle (outside all timing; the
    # batch-8 config-5 line shares frame 0's seed with the batch-1 line, checked once)
    pyoracle.lib()
    verdict = {}

    def work(item):
        name, (L0, R0), got, fn = item
        if fn is not None:
            verdict[name] = bool(np.array_equal(got, fn(L0, R0)))

    ts = [threading.Thread(target=work, args=(c,)) for c in checks]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for name, rec in recs.items():
        rec["parity_frame0"] = verdict.get(name, verdict.get(name.replace("batch8", "batch1")))
    return recs


def cpu_info():
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    return {"nproc": os.cpu_count(), "affinity": aff, "model": model}


def cpu_baseline(frames, params, threads):
    """Oracle (scalar C restatement of OpenCV 3.4, 'port') on host cores, one frame per thread."""
    from oracle import pyoracle
    pyoracle.lib()
    p = {k: v for k, v in params.items() if k != "variant"}
    outs = [None] * len(frames)
    nxt = [0]
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(frames):
                return
            L, R = frames[i]
            outs[i] = pyoracle.sgbm(L, R, p)  # ctypes releases the GIL

    t0 = time.perf_counter()
    ts = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return time.perf_counter() - t0, outs


def dry_main(args, world, rank):
    """Launcher + gather rehearsal: gloo ranks, host frames, out = L - R (int16)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd.batch import FrameBatch, frame_seeds
    if world > 1:
        dist.init_process_group("gloo")
    W, H, F = args.width, args.height, args.frames
    seeds = frame_seeds(rank, world, F, SEED0)
    pairs = [mvsv.synth_pair(sd, W, H, 0, 16) for sd in seeds]
    L = torch.from_numpy(np.stack([p[0] for p in pairs]))
    R = torch.from_numpy(np.stack([p[1] for p in pairs]))
    out = torch.empty((F, H, W), dtype=torch.int16)

    def compute(Lb, Rb, o):
        o.copy_(Lb.to(torch.int16) - Rb.to(torch.int16))

    batch = FrameBatch(L, R, out, compute, rank, world, gather=world > 1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        got = batch.step()
    elapsed = time.perf_counter() - t0
    if rank == 0:
        got = torch.cat(got) if world > 1 else out
        ok = 0
        for r in range(world):
            for j, sd in enumerate(frame_seeds(r, world, F, SEED0)):
                Lh, Rh = mvsv.synth_pair(sd, W, H, 0, 16)
                ok += int(np.array_equal(got[r * F + j].numpy(),
                                         Lh.astype(np.int16) - Rh.astype(np.int16)))
        print(json.dumps({"dry": True, "n_gpus": world, "global_batch": F * world,
                          "gather": "gloo" if world > 1 else "none",
                          "gathered_frames_ok": f"{ok}/{F * world}",
                          "ms_per_step": round(elapsed / max(args.steps, 1) * 1e3, 3)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main(argv=None):
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.force_gather):
        return launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        return 2
    if args.dry:
        return dry_main(args, world, rank)

    import numpy as np
    import torch
    import torch.distributed as dist

    import mvstereovision3_amd as mvsv
    from mvstereovision3_amd import _lib

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or args.force_gather
    out_fd = None
    if distributed:
        # RCCL prints its banner (and any library chatter) on stdout: keep the
        # process's stdout for the one JSON line and send everything else to
        # stderr
        sys.stdout.flush()
        out_fd = os.dup(1)
        os.dup2(2, 1)
        dist.init_process_group("nccl", device_id=dev)

    W, H, F = args.width, args.height, args.frames
    m = mvsv.StereoSGBM.create(0, 0, 0, 8 * 0 * 0, 32 * 0 * 0)  # trgt/mean_test.cpp:233-237
    para = mvsv.sgbmParameters()
    assert mvsv.Disparity.loadSGBMParameters(SGBM_YML, m, para), "cannot load sgbm.yml"
    m.setMode(args.mode)
    params = m.params()
    D, minD = params["num_disparities"], params["min_disparity"]
    W1 = W - max(minD + D, 0) + min(minD, 0)
    ndir = 8 if args.mode == 1 else 5
    P1 = params["p1"] if params["p1"] > 0 else 2
    P2 = max(params["p2"] if params["p2"] > 0 else 5, P1 + 1)
    # bytes per (pixel, disparity) of an accumulator plane: 4-bit planes on the
    # strip schedule when 3 * P2 <= 15 (sgbm.yml: P2 = 5), else u8 / u16
    acc = 0.5 if (D in (32, 64, 128, 256) and 3 * P2 <= 15) else (1 if ndir * P2 <= 255 else 2)
    # the pipeline the library will run for this launch, as it reports it
    # (mvsv_sgbm_plan): bit-sliced (MODE_HH or MODE_SGBM, sgbm.yml's regime),
    # side by side or strips, the nibble residual plane of the packed passes
    plan = _lib.sgbm_plan(_lib.context(dev.index or 0), F, W, H, m._params)
    bitslice = bool(plan & _lib.PLAN_BITSLICE)
    side = bool(plan & _lib.PLAN_SIDE)
    residual = bool(plan & _lib.PLAN_RESIDUAL)

    from mvstereovision3_amd.batch import FrameBatch, InflightBatches, frame_seeds
    host = [mvsv.synth_pair(sd, W, H, minD, D) for sd in frame_seeds(rank, world, F, SEED0)]
    Lt = torch.from_numpy(np.stack([h[0] for h in host])).to(dev)
    Rt = torch.from_numpy(np.stack([h[1] for h in host])).to(dev)
    gather = distributed and not args.no_gather
    compute = lambda L, R, o: m.compute(L, R, o)  # noqa: E731
    n_in = max(1, args.inflight)
    if n_in > 1:
        batch = InflightBatches(Lt, Rt, lambda: torch.empty((F, H, W), dtype=torch.int16, device=dev),
                                compute, n_in, dev, rank, world, gather, collective=args.force_gather)
        out = batch.slots[0][2]
        contexts = batch.contexts()
    else:
        out = torch.empty((F, H, W), dtype=torch.int16, device=dev)
        batch = FrameBatch(Lt, Rt, out, compute, rank, world, gather, collective=args.force_gather)
        contexts = [_lib.context(local)]

    def check_contexts():
        # raises if a launch of these steps gave up a strip hand-off (maps INVALID)
        for c in contexts:
            _lib.check(_lib.lib().mvsv_synchronize(c.handle), c.handle)

    def barrier():
        torch.cuda.synchronize(dev)
        if distributed:
            dist.barrier(device_ids=[local])
        torch.cuda.synchronize(dev)

    warm = max(args.warmup, n_in)  # every slot's buffers allocated before timing
    for _ in range(warm):
        batch.step()
    barrier()
    check_contexts()
    K = args.steps
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(K):
        batch.step()
        if n_in == 1:
            ev[i + 1].record()
    barrier()
    t1 = time.perf_counter()
    check_contexts()  # no map of the timed steps came from a given-up hand-off
    elapsed = t1 - t0
    step_ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(K)] if n_in == 1 else None
    # stage times for the roofline: a separate pass, one step after the other
    # on the default context (with batches in flight the launches overlap, so
    # their spans are not kernel durations)
    ctx = _lib.context(local)
    pout = torch.empty((F, H, W), dtype=torch.int16, device=dev)
    compute(Lt, Rt, pout)
    barrier()
    _lib.profile_reset(ctx)
    _lib.profile_enable(ctx, True)
    P = max(1, args.profile_steps)
    p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    p0.record()
    for _ in range(P):
        compute(Lt, Rt, pout)
    p1.record()
    barrier()
    _lib.profile_enable(ctx, False)
    prof = _lib.profile_read(ctx)
    _lib.synchronize(local)
    single_ms = p0.elapsed_time(p1) / P
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the gathered global batch of the last timed step, on rank 0 (host copy,
    # outside the timed region) for the parity sample below
    gathered = None
    if gather and rank == 0 and batch.gathered is not None:
        gathered = [g.cpu().numpy() for g in batch.gathered]

    if rank == 0:
        ms_per_step = elapsed / K * 1e3
        mpix = world * F * W * H * K / elapsed / 1e6
        stages = {k: {"ms_per_step": v[0] / P, "launches_per_step": v[1] / P}
                  for k, v in prof.items() if v[1]}
        strips = D in (32, 64, 128, 256)
        # dominant KERNEL: path_aggregation is the span of the strip and line
        # kernels (which run concurrently) when both are timed separately
        kernels = [k for k in stages if not (k == "path_aggregation" and "path_strips" in stages)]
        dom = max(kernels, key=lambda k: stages[k]["ms_per_step"])
        launches = stages[dom]["launches_per_step"]
        avg_launch_s = stages[dom]["ms_per_step"] / launches / 1e3
        # SURVEY.md §8(d) compulsory bytes per frame (8 paths): u8 L+R in, int16
        # map out, one int16 write + read of the cross-sweep aggregate per (px, d)
        comp = 4 * W * H * (1 + D)
        alg_bytes_per_launch = comp * F / launches
        achieved = alg_bytes_per_launch / avg_launch_s / 1e9
        impl_bytes_per_launch = stage_bytes(dom, F, W, H, W1, D, ndir, acc, strips, residual, bitslice,
                                            side) / launches
        workload = f"sgbm_{W}x{H}_d{D}_{ndir}path_batch{F}"
        sha = kernel_source_sha()
        pmc, traffic_note = _summary(PMC_FILE, workload, sha, "PMC")
        traffic = pmc.get("stages", {}).get(dom, {}).get("hbm_bytes_per_launch") if pmc else None
        if pmc:
            traffic_note += " (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE in separate passes)"
        sq, sq_note = _summary(SQ_FILE, workload, sha, "SQ")
        valu_frac = sq.get("stages", {}).get(dom, {}).get("valu_util") if sq else None
        if sq:
            sq_note += " (rocprofv3 SQ_ACTIVE_INST_VALU x4 / (1024 SIMDs x GRBM_GUI_ACTIVE/8))"
        # measured HBM utilisation of the dominant kernel: counter bytes over its
        # live launch time, against the same peak
        hbm_util = traffic / avg_launch_s / 1e9 / HBM_PEAK_GBPS if traffic else None
        if valu_frac is not None and hbm_util is not None:
            bound = "valu" if valu_frac > hbm_util else "hbm"
        else:
            bound = "unmeasured"
        res = {
            "metric": "Mpix disparities/sec (SGBM 128-disp, 8-path) at 1/2/4/8 GPUs; % HBM roofline",
            "value": round(mpix, 2),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "median_ms_per_step": round(statistics.median(step_ms), 4) if step_ms else None,
            "inflight": n_in,
            "single_batch_ms": round(single_ms, 4),
            "single_batch_mpix_s": round(F * W * H / single_ms / 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16",
            "data": "synthetic (PCG32 rectified pairs, SURVEY.md §8(d)), HBM-resident",
            "config": {"workload": f"sgbm_{W}x{H}_d{D}_{ndir}path_batch{F}",
                       "width": W, "height": H, "num_disparities": D, "min_disparity": minD,
                       "block_size": params["block_size"], "mode": "MODE_HH" if args.mode == 1 else "MODE_SGBM",
                       "paths": ndir, "frames_per_gpu": F, "global_batch": F * world,
                       "params": "configs/sgbm.yml + mode", "gather": "rccl" if gather else "none",
                       "launch": "torch.distributed.run" if distributed else "single process",
                       "batches_in_flight": n_in,
                       "parallelism": f"frame-parallel x{world}"},
            "roofline": {"kernel": dom, "bound": bound,
                         "bound_rule": "larger of the measured utilisations hbm_util (PMC traffic) and "
                                       "valu_frac (SQ counters) of the dominant kernel",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "traffic_source": traffic_note,
                         "hbm_util": round(hbm_util, 4) if hbm_util is not None else None,
                         "valu_frac": valu_frac,
                         "valu_source": sq_note,
                         "pipeline_frac": round(comp * F * K / elapsed / 1e9 / HBM_PEAK_GBPS, 5),
                         "pipeline_frac_rule": "SURVEY.md §8(d) bytes of the whole step over its wall time / peak",
                         "algorithmic_bytes_per_launch": int(alg_bytes_per_launch),
                         "algorithmic_bytes": "SURVEY.md §8(d): 4*W*H*(1+D) per frame x frames per launch",
                         "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                         "impl_bytes_per_launch": int(impl_bytes_per_launch),
                         "impl_frac": round(impl_bytes_per_launch / avg_launch_s / 1e9 / HBM_PEAK_GBPS, 4)},
            "pipeline_compulsory": {"bytes_per_frame": comp,
                                    "achieved_GBps_per_gpu": round(comp * F * K / elapsed / 1e9, 1),
                                    "frac_of_peak": round(comp * F * K / elapsed / 1e9 / HBM_PEAK_GBPS, 5)},
            "stages_ms_per_step": {k: round(v["ms_per_step"], 4) for k, v in stages.items()},
            "stages_source": f"HIP events around each stage, {P} steps one after the other (no overlap)",
        }
        if world == 1 and not args.no_cpu_baseline:
            info = cpu_info()
            thr = args.cpu_threads or max(1, min(CPU_SHARE, info["affinity"]))
            # one frame per thread: the first F are the GPU's frames (parity sample)
            seeds = [SEED0 + i for i in range(thr)]
            frames = [host[i] if i < F else mvsv.synth_pair(seeds[i], W, H, minD, D)
                      for i in range(thr)]
            wall, ref = cpu_baseline(frames, params, thr)
            lat, _ = cpu_baseline(frames[:1], params, 1)
            nchk = min(F, thr)
            gpu_out = out[:nchk].cpu().numpy()
            same = sum(int(np.array_equal(gpu_out[i], ref[i])) for i in range(nchk))
            res["cpu_baseline"] = {"value": round(thr * W * H / wall / 1e6, 3), "unit": "Mpix/s",
                                   "cores": thr, "kind": "port",
                                   "sample": f"{thr} frames of the same workload, one frame per "
                                             f"thread on {thr} threads, scalar C oracle (OpenCV "
                                             f"3.4 restatement, no SIMD -- slower than OpenCV's "
                                             f"SSE2 path), {wall:.1f} s wall",
                                   "latency_1core_s": round(lat, 3),
                                   "host": info}
            res["parity_sample"] = f"{same}/{nchk} frames bit-exact vs oracle"
        if world == 1 and not args.no_configs and not distributed:
            tc0 = time.perf_counter()
            res["configs"] = config_table(mvsv, _lib, dev)
            res["configs_note"] = (f"BASELINE configs 1, 2, 3, 5 on this GPU, device-resident (median of 10 "
                                   f"HIP-event steps after 3 warm-up), roof per SURVEY.md §8(d), parity_frame0 = "
                                   f"frame 0 vs the oracle; {time.perf_counter() - tc0:.1f} s incl. oracles")
        if gathered is not None:
            # the gathered global batch: frame 0 of every rank, as it arrived on
            # rank 0, against the oracle (outside the timed region)
            sample = [(r, mvsv.synth_pair(frame_seeds(r, world, F, SEED0)[0], W, H, minD, D))
                      for r in range(world)]
            thr = max(1, min(CPU_SHARE, cpu_info()["affinity"], world))
            _, ref = cpu_baseline([p for _, p in sample], params, thr)
            ok = sum(int(np.array_equal(gathered[r][0], ref[i])) for i, (r, _) in enumerate(sample))
            res["parity_sample_gathered"] = (f"{ok}/{world} gathered frames (frame 0 of each rank, "
                                             f"received on rank 0 through dist.gather) bit-exact vs oracle")
        line = json.dumps(res)
        if out_fd is not None:
            sys.stdout.flush()
            os.write(out_fd, (line + "\n").encode())
        else:
            print(line, flush=True)
    if distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
