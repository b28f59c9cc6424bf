"""No scratch in the kernels the pipelines dispatch (CPU test on the built library).

Reads the AMDGPU kernel metadata of the gfx950 code objects embedded in
mvstereovision3_amd/libmvsv.so (.hip_fatbin -> clang offload bundles -> ELF
notes) and checks `.private_segment_fixed_size` == 0 for every kernel of the
bit-sliced SGBM step (sgbm.yml, MODE_HH) and its cost kernel: a spilled kernel
sends its spills through scratch, whose evicted lines reach HBM (round 5 found
the blockSize-13 cost kernel spilling 48 VGPRs: 0.6 GB of extra writes per
8-frame step; DESIGN.md round-5 summary).  tools/kernel_resources.py lists
every kernel's registers and scratch from the compiler's remarks.

Round 6: every kernel instance that BASELINE configs 1-5 and the reference's
call sites (liveDisparity create(0, 64 | 256, 9, 648, 2592), captureDisparity
create(0, 16, 5, 200, 800)) dispatch at batches of 1, 2 and 8 frames --
recorded on the GPU by tools/gpu_census.sh into tests/golden/dispatch_census.json
-- must carry no scratch either.
"""
import json
import os
import re
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mvstereovision3_amd", "libmvsv.so")
LLVM = "/opt/rocm/lib/llvm/bin"

HEADLINE = [r"bsgm_", r"sgbm_cost2_kernelILi13ELi1ELi64E", r"sgbm_prefilter_kernel",
            r"median3x3_pk_kernel", r"speckle_"]


def kernel_scratch():
    """{mangled kernel name: private segment bytes} over every gfx950 code object."""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB,
                        os.path.join(td, "x.so")], check=True, capture_output=True)
        b = open(fat, "rb").read()
        out = {}
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        i = b.find(magic)
        while i >= 0:
            n = struct.unpack_from("<Q", b, i + len(magic))[0]
            p = i + len(magic) + 8
            for _ in range(n):
                off, size, tl = struct.unpack_from("<QQQ", b, p)
                p += 24
                triple = b[p:p + tl].decode()
                p += tl
                if "gfx950" in triple and size:
                    co = os.path.join(td, "dev.co")
                    open(co, "wb").write(b[i + off:i + off + size])
                    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                                           capture_output=True, text=True).stdout
                    name = None
                    for line in notes.splitlines():
                        m = re.match(r"\s+\.name:\s+(\S+)", line)
                        if m:
                            name = m.group(1)
                        m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
                        if m and name:
                            out[name] = int(m.group(1))
            i = b.find(magic, i + 1)
        return out


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(f"{LLVM}/llvm-readelf"),
                    reason="library not built / no ROCm llvm tools")
def test_headline_kernels_have_no_scratch():
    ks = kernel_scratch()
    assert len(ks) > 20, "no kernel metadata found in the library"
    picked = {k: v for k, v in ks.items() if any(re.search(p, k) for p in HEADLINE)}
    for p in HEADLINE:
        assert any(re.search(p, k) for k in picked), f"no kernel matches {p}"
    bad = {k: v for k, v in picked.items() if v}
    assert not bad, f"headline kernels with scratch: {bad}"


CENSUS = os.path.join(ROOT, "tests", "golden", "dispatch_census.json")


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(f"{LLVM}/llvm-readelf"),
                    reason="library not built / no ROCm llvm tools")
def test_dispatched_kernels_have_no_scratch():
    ks = kernel_scratch()
    names = list(ks)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    by_name = dict(zip(dem, names))
    census = json.load(open(CENSUS))["configs"]
    assert set(census) >= {"c1", "c2", "c3m0", "c3m1", "c4", "c5", "live64", "capture"}
    bad, missing = {}, []
    for cfg, kernels in census.items():
        for k in kernels:
            m = by_name.get(k)
            if m is None:
                missing.append((cfg, k))
            elif ks[m]:
                bad[k] = (cfg, ks[m])
    assert not missing, f"census kernels not in the library (re-run tools/gpu_census.sh): {missing[:5]}"
    assert not bad, f"dispatched kernels with scratch: {bad}"
