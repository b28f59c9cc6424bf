#!/usr/bin/env python3
"""Summarise an MVSV_TRI_TRACE file of the sheared-strip kernel.

Per strip and step the kernel records (100 MHz clock, comparable across CUs)
when the step's boundary granules went out (publish) and when the producer's
step was in (consume).  Prints, over the strips of chain 0: the hop latency
(consume of step t by strip k - publish of step t by strip k-1), the step
interval of the publishing side, and the start / end of every 8th strip.

    python tools/tri_trace.py TRACE_FILE
"""
import sys

import numpy as np


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64)
    nblk, sb, H, nstrips, npass, nfr, sw, w1 = (int(v) for v in raw[:8])
    d = raw[8:].reshape(nblk, sb).astype(np.int64)
    pub = d[:, 8:8 + H]
    got = d[:, 8 + H:8 + 2 * H]
    nch = npass * nfr
    print(f"blocks {nblk} strips {nstrips} chains {nch} H {H} strip width {sw} W1 {w1}")
    hops, steps = [], []
    t_first = pub[pub > 0].min()
    for k in range(nstrips):
        b = k * nch
        if b >= nblk:
            break
        live = pub[b] > 0
        if not live.any():
            continue
        ts = np.nonzero(live)[0]
        p = pub[b, ts]
        steps.extend(np.diff(p).tolist())
        if k > 0:
            bp = (k - 1) * nch
            both = (got[b] > 0) & (pub[bp] > 0)
            hops.extend((got[b, both] - pub[bp, both]).tolist())
        if k % 8 == 0:
            print(f"strip {k:4d}: steps {ts[0]}..{ts[-1]}, first publish +{(p[0] - t_first) / 100:.1f} us, "
                  f"last +{(p[-1] - t_first) / 100:.1f} us, {(p[-1] - p[0]) / max(len(ts) - 1, 1) * 10:.0f} ns/step")
    hops = np.array(hops) * 10
    steps = np.array(steps) * 10
    q = [10, 50, 90, 99]
    print("hop ns (consume k - publish k-1, same step) p10/50/90/99:", np.percentile(hops, q).round().tolist())
    print("step interval ns p10/50/90/99:", np.percentile(steps, q).round().tolist())
    print(f"span {(pub.max() - t_first) / 100:.1f} us")


if __name__ == "__main__":
    main()
