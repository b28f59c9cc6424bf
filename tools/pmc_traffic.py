#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE collected in
separate runs, MI355X_MICROARCH.md §HBM) into per-stage HBM bytes per launch.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv WORKLOAD OUT.json

gfx950 corrections (MI355X_MICROARCH.md): FETCH_SIZE is in KiB and reports half
the bytes of a wide coalesced streaming read -> fetch_bytes = 2 * FETCH_SIZE *
1024 ("corrected"); WRITE_SIZE (KiB) is exact for streaming stores.  Both the
raw and the corrected values are written; bench.py uses the corrected total.
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_source_sha  # noqa: E402

STAGES = [("sgbm_tri_kernel", "path_strips"), ("bsgm_strip_kernel", "path_strips"),
          ("bsgm_lines4_kernel", "path_lines"), ("bsgm_wta_kernel", "final_wta_lr"),
          ("bsgm_rlwta_kernel", "final_wta_lr"), ("bsgm_rl_final_kernel", "final_wta_lr"),
          ("bsgm_dir_kernel", "path_aggregation"),
          ("sgbm_path16_kernel", "path_lines"),
          ("sgbm_path_kernel", "path_aggregation"), ("sgbm_cost_fixup", "cost_fixup"),
          ("sgbm_cost", "cost_volume"), ("sgbm_final", "final_wta_lr"),
          ("sgbm_prefilter", "prefilter"), ("median3x3", "post_filters"),
          ("speckle", "post_filters"), ("bm_match", "bm_match")]


def stage_of(name):
    for key, st in STAGES:
        if key in name:
            return st
    return None


def per_dispatch(path, counter):
    vals = defaultdict(float)
    names = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r.get("Counter_Name") != counter:
                continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            vals[d] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    return vals, names


def main(fetch_csv, write_csv, workload, out):
    f, fn = per_dispatch(fetch_csv, "FETCH_SIZE")
    w, wn = per_dispatch(write_csv, "WRITE_SIZE")
    # a stage's launches = the dispatch count of its most frequent kernel (one
    # per step), so a stage of several kernels (post filters, the fused R->L +
    # WTA and its finishing pass) reports its bytes per step
    acc = defaultdict(lambda: {"launches": 0, "fetch_kib": 0.0, "per_kernel": defaultdict(int)})
    accw = defaultdict(lambda: {"launches": 0, "write_kib": 0.0, "per_kernel": defaultdict(int)})
    for d, v in f.items():
        st = stage_of(fn[d])
        if st:
            acc[st]["per_kernel"][fn[d]] += 1
            acc[st]["launches"] = max(acc[st]["per_kernel"].values())
            acc[st]["fetch_kib"] += v
    for d, v in w.items():
        st = stage_of(wn[d])
        if st:
            accw[st]["per_kernel"][wn[d]] += 1
            accw[st]["launches"] = max(accw[st]["per_kernel"].values())
            accw[st]["write_kib"] += v
    stages = {}
    for st in sorted(set(acc) | set(accw)):
        fl = acc[st]["launches"] or 1
        wl = accw[st]["launches"] or 1
        fetch = acc[st]["fetch_kib"] / fl * 1024
        write = accw[st]["write_kib"] / wl * 1024
        stages[st] = {"launches_fetch_pass": acc[st]["launches"],
                      "launches_write_pass": accw[st]["launches"],
                      "fetch_bytes_raw_per_launch": int(fetch),
                      "write_bytes_per_launch": int(write),
                      "hbm_bytes_per_launch": int(2 * fetch + write),
                      "hbm_bytes_per_launch_uncorrected": int(fetch + write)}
    json.dump({"workload": workload, "source": [fetch_csv, write_csv],
               "kernel_source_sha": kernel_source_sha(),
               "correction": "fetch x2 (gfx950 FETCH_SIZE halving for wide streaming reads)",
               "stages": stages}, open(out, "w"), indent=1)
    print(json.dumps(stages, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
