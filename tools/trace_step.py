"""Print the kernels of the last pipeline step of a rocprofv3 kernel trace."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seq = []
for r in rows:
    k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0].split("::")[-1]
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    seq.append((k, t, r["Grid_Size_X"], r["Grid_Size_Y"], r["VGPR_Count"], r["LDS_Block_Size"]))
starts = [i for i, s in enumerate(seq) if s[0].startswith("sgbm_prefilter")]
a = starts[-1]
b = len(seq)
tot = 0.0
for k, t, gx, gy, v, l in seq[a:b]:
    tot += t
    print(f"{k:52s} {t:9.1f} us  grid {gx}x{gy} vgpr {v} lds {l}")
print(f"total {tot:.1f} us")
