"""Timings of the StereoBM match kernels (run on the box: python tools/bm_time.py): configs 1 / 2 at
batch 1 and 8, the disparities-on-lanes kernel with the chosen tile height and
a sweep of MVSV_BM_TY, then the 16x16-tile kernel (MVSV_KERNELS=bm-tile)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mvstereovision3_amd as mvsv  # noqa: E402
from mvstereovision3_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
CASES = (("config2", 64, 9, None), ("config1", 80, 21, "tests/golden/configs/bm.yml"))


def run(tag, cases=CASES, batches=(1, 8)):
    _lib._tls.ctxs = {}
    for name, D, bs, yml in cases:
        b = mvsv.StereoBM.create(D, bs)
        if yml:
            mvsv.Disparity.loadBMParameters(yml, b)
        for n in batches:
            pairs = [mvsv.synth_pair(0x5EED0000 + i, 640, 480, 0, D) for i in range(n)]
            L = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
            R = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
            out = torch.empty((n, 480, 640), dtype=torch.int16, device=dev)
            for _ in range(3):
                b.compute(L, R, out)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                b.compute(L, R, out)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 20
            print(f"{tag:10s} {name} n={n} {dt * 1e3:.3f} ms {n * 640 * 480 / dt / 1e6:.0f} Mpix/s", flush=True)


if len(sys.argv) > 1 and sys.argv[1] == "--one":  # --one NAME N: one case (counter passes)
    case = [c for c in CASES if c[0] == sys.argv[2]]
    run("one", cases=case, batches=(int(sys.argv[3]),))
    sys.exit(0)
run("auto")
if len(sys.argv) > 1 and sys.argv[1] == "--auto":  # the chosen tile height only (A/B runs)
    sys.exit(0)
for ty in (8, 12, 16, 20):
    os.environ["MVSV_BM_TY"] = str(ty)
    run(f"ty={ty}", batches=(8,))
os.environ.pop("MVSV_BM_TY")
os.environ["MVSV_KERNELS"] = "bm-tile"
run("tile")
