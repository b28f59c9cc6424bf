#!/usr/bin/env python3
"""Per-kernel / per-stage summary of the SQ + GRBM counter passes written by
tools/sq_counters.sh (rocprofv3 --pmc, one pass per counter group).

    python tools/sq_summary.py DIR [WORKLOAD OUT.json]

Counter units (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units"):
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over
waves; GRBM_GUI_ACTIVE counts GPU cycles summed over the 8 XCDs.  Per dispatch:

  kernel_cycles = GRBM_GUI_ACTIVE / 8          (the dispatch's duration, cycles)
  valu_util     = 4 * SQ_ACTIVE_INST_VALU / (SIMDs * kernel_cycles)
                  the fraction of SIMD cycles in which some wave of that SIMD
                  was issuing a vector instruction (the waves of a SIMD issue
                  VALU one at a time, so their active cycles add)
  valu_cyc_per_inst = 4 * SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU
  issue / parked / stalled = SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY / SQ_WAIT_INST_ANY
                  as fractions of SQ_WAVE_CYCLES (disjoint)
  lds_util      = SQ_LDS_IDX_ACTIVE / (CUs * kernel_cycles)

The JSON carries the kernel-source sha (bench.py's kernel_source_sha) so a
summary of other sources is never quoted as this build's.
"""
import collections
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CUS = 256
SIMDS = 4 * CUS
XCDS = 8

STAGES = [("sgbm_tri_kernel", "path_strips"), ("bsgm_strip_kernel", "path_strips"),
          ("bsgm_lines4_kernel", "path_lines"), ("bsgm_wta_kernel", "final_wta_lr"),
          ("bsgm_rlwta_kernel", "final_wta_lr"), ("bsgm_rl_final_kernel", "final_wta_lr"),
          ("bsgm_dir_kernel", "path_aggregation"),
          ("sgbm_path16_kernel", "path_lines"),
          ("sgbm_pathdirs16_kernel", "path_aggregation"), ("sgbm_path_kernel", "path_aggregation"),
          ("sgbm_cost_fixup", "cost_fixup"), ("sgbm_cost", "cost_volume"),
          ("sgbm_final", "final_wta_lr"), ("sgbm_prefilter", "prefilter"),
          ("median3x3", "post_filters"), ("speckle", "post_filters"), ("bm_match", "bm_match")]


def kname(s):
    s = s.replace("(anonymous namespace)::", "")
    return re.split(r"[(<]", s)[0].split("::")[-1]


def stage_of(name):
    for key, st in STAGES:
        if key in name:
            return st
    return None


def find_csv(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return os.path.join(root, f)
    raise FileNotFoundError(f"no counter_collection.csv under {d}")


def load(d):
    """{dispatch: {counter: value}} and {dispatch: kernel name} over both passes.
    Dispatch ids differ between passes, so passes are matched by kernel name
    and order of occurrence."""
    per = []
    for pas in ("p1", "p2"):
        rows = collections.OrderedDict()
        for r in csv.DictReader(open(find_csv(os.path.join(d, pas)))):
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            e = rows.setdefault(key, {"name": r["Kernel_Name"], "c": collections.defaultdict(float),
                                      "vgpr": float(r.get("VGPR_Count") or 0),
                                      "lds": float(r.get("LDS_Block_Size") or 0)})
            e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
        per.append(list(rows.values()))
    # match by (kernel name, occurrence index)
    merged = []
    seen = collections.Counter()
    idx2 = collections.defaultdict(list)
    for e in per[1]:
        idx2[e["name"]].append(e)
    for e in per[0]:
        k = e["name"]
        j = seen[k]
        seen[k] += 1
        c = dict(e["c"])
        if j < len(idx2[k]):
            for n, v in idx2[k][j]["c"].items():
                if n not in c:
                    c[n] = v
        merged.append({"name": k, "c": c, "vgpr": e["vgpr"], "lds": e["lds"]})
    return merged


def summarize(disp):
    agg = collections.OrderedDict()
    for e in disp:
        k = kname(e["name"])
        a = agg.setdefault(k, {"n": 0, "c": collections.defaultdict(float), "vgpr": e["vgpr"],
                               "lds": e["lds"], "stage": stage_of(k)})
        a["n"] += 1
        for n, v in e["c"].items():
            a["c"][n] += v
    out = collections.OrderedDict()
    for k, a in agg.items():
        c = a["c"]
        n = a["n"]
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / XCDS / n
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1.0
        valu = c.get("SQ_ACTIVE_INST_VALU", 0) / n
        iv = c.get("SQ_INSTS_VALU", 0) / n
        out[k] = {
            "stage": a["stage"], "dispatches": n, "vgpr": a["vgpr"], "lds_bytes": a["lds"],
            "kernel_cycles": round(cyc),
            "valu_insts": iv,
            "valu_util": round(4 * valu / (SIMDS * cyc), 4) if cyc else None,
            "valu_cyc_per_inst": round(4 * valu / iv, 3) if iv else None,
            "valu_issue_per_simd_cycle": round(iv / (SIMDS * cyc), 4) if cyc else None,
            "issue": round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
            "parked_waitcnt_barrier": round(c.get("SQ_WAIT_ANY", 0) / wc, 4),
            "stalled_issue": round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
            "lds_issue_stall": round(c.get("SQ_WAIT_INST_LDS", 0) / wc, 4),
            "lds_util": round(c.get("SQ_LDS_IDX_ACTIVE", 0) / n / (CUS * cyc), 4) if cyc else None,
            "lds_bank_conflict_frac": round(c.get("SQ_LDS_BANK_CONFLICT", 0) / (c.get("SQ_LDS_IDX_ACTIVE", 0) or 1), 4),
            "insts_per_dispatch": {x: c.get(f"SQ_INSTS_{x.upper()}", 0) / n
                                   for x in ("valu", "salu", "lds", "vmem_rd", "vmem_wr")},
            "waves_per_dispatch": c.get("SQ_WAVES", 0) / n,
        }
    return out


def main(d, workload=None, out=None):
    s = summarize(load(d))
    for k, v in s.items():
        print(f"{k} [{v['stage']}] x{v['dispatches']}: {v['kernel_cycles']} cyc, VALU util {v['valu_util']} "
              f"({v['valu_cyc_per_inst']} cyc/inst), issue {v['issue']} parked {v['parked_waitcnt_barrier']} "
              f"stalled {v['stalled_issue']}, LDS util {v['lds_util']} (conflicts {v['lds_bank_conflict_frac']}), "
              f"VGPR {v['vgpr']:.0f}")
    if out:
        from bench import kernel_source_sha
        stages = collections.OrderedDict()
        for k, v in s.items():
            st = v["stage"]
            if not st:
                continue
            a = stages.setdefault(st, {"kernels": [], "kernel_cycles": 0, "valu_busy_cycles": 0.0})
            a["kernels"].append(k)
            a["kernel_cycles"] += v["kernel_cycles"]
            if v["valu_util"] is not None:
                a["valu_busy_cycles"] += v["valu_util"] * v["kernel_cycles"]
        for a in stages.values():
            a["valu_util"] = round(a["valu_busy_cycles"] / a["kernel_cycles"], 4) if a["kernel_cycles"] else None
        json.dump({"workload": workload, "kernel_source_sha": kernel_source_sha(),
                   "units": __doc__.split("Counter units")[1].split("The JSON")[0].strip(),
                   "kernels": s, "stages": stages}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:4])
