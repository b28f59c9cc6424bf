#!/usr/bin/env python3
"""Register / scratch audit of the HIP kernels: compiles each source for gfx950
with -Rpass-analysis=kernel-resource-usage and prints every kernel's VGPRs,
spilled VGPRs and scratch bytes per lane (a spilled kernel sends its spills
through the vector memory path: scratch loads park the wave, and evicted
scratch lines reach HBM as WRITE_SIZE the algorithm does not account for).

    python tools/kernel_resources.py [--filter REGEX] [--all] [-D NAME=VAL ...] [FILES...]

Without --all only kernels with scratch are listed.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mvstereovision3_amd", "csrc")
DEFAULT = ["mvsv_cost.hip", "mvsv_sgbm.hip", "mvsv_bsgm.hip", "mvsv_bm.hip", "mvsv_post.hip"]


def demangle(names):
    try:
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(names),
                             capture_output=True, text=True, check=True).stdout.splitlines()
        return [o.replace("mvsv::(anonymous namespace)::", "") for o in out]
    except Exception:
        return names


def audit(src, defines):
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
               "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "--cuda-device-only", "-x", "hip",
               "-c", os.path.join(CSRC, src), "-o", os.path.join(td, "k.co"),
               "-Rpass-analysis=kernel-resource-usage"] + ["-D" + d for d in defines]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode:
            sys.exit(p.stderr[-4000:])
    rows, cur = [], None
    for line in p.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r"remark:\s+VGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"),
                         ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
    for r, d in zip(rows, demangle([r["name"] for r in rows])):
        r["name"] = d
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="*", default=DEFAULT)
    ap.add_argument("--filter", default="")
    ap.add_argument("--all", action="store_true")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args()
    for f in a.files:
        for r in audit(f, a.defines):
            if a.filter and not re.search(a.filter, r["name"]):
                continue
            if a.all or r.get("scratch", 0) > 0:
                print(f"{f}: {r['name'][:110]}  vgpr {r.get('vgpr')} spill {r.get('spill')} "
                      f"scratch {r.get('scratch')} occ {r.get('occ')}")


if __name__ == "__main__":
    main()
