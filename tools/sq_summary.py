"""Per-kernel averages of SQ counter passes (tools/sq_counters.sh output)."""
import collections
import csv
import re
import sys


def kname(s):
    s = s.replace("(anonymous namespace)::", "")
    return re.split(r"[(<]", s)[0].split("::")[-1]


def main(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for pas in ("p1", "p2"):
        for r in csv.DictReader(open(f"{d}/{pas}/run_counter_collection.csv")):
            k = kname(r["Kernel_Name"])
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            agg[k]["VGPR"] = [float(r["VGPR_Count"])]
            agg[k]["LDS"] = [float(r["LDS_Block_Size"])]
    for k, c in agg.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"{k}: VGPR {m['VGPR']:.0f} LDS {m['LDS']:.0f} waves {m.get('SQ_WAVES', 0):.0f} "
              f"busy {m.get('SQ_BUSY_CYCLES', 0):.3g}")
        print(f"   wave_cycles {wc:.3g}: active {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
              f"wait_any {m.get('SQ_WAIT_ANY', 0) / wc:.2f} wait_inst {m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
              f"(lds issue {m.get('SQ_WAIT_INST_LDS', 0) / wc:.2f})")
        print(f"   insts valu {m.get('SQ_INSTS_VALU', 0):.3g} lds {m.get('SQ_INSTS_LDS', 0):.3g} "
              f"salu {m.get('SQ_INSTS_SALU', 0):.3g} vmem rd {m.get('SQ_INSTS_VMEM_RD', 0):.3g} "
              f"wr {m.get('SQ_INSTS_VMEM_WR', 0):.3g}; lds bank-conflict/idx-active "
              f"{m.get('SQ_LDS_BANK_CONFLICT', 0):.3g}/{m.get('SQ_LDS_IDX_ACTIVE', 0):.3g}")


if __name__ == "__main__":
    main(sys.argv[1])
