#!/bin/bash
# Disassemble one source's gfx950 device code: tools/disasm.sh mvsv_cost.hip [out.s] [-DNAME=V ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
SRC=${1:?source in mvstereovision3_amd/csrc}; OUT=${2:-/tmp/$(basename $SRC .hip).s}; shift 2 || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/include -I$R/mvstereovision3_amd/csrc \
  --cuda-device-only --no-gpu-bundle-output -x hip -c $R/mvstereovision3_amd/csrc/$SRC -o /tmp/disasm_$$.co "$@"
/opt/rocm/llvm/bin/llvm-objdump -d /tmp/disasm_$$.co > $OUT
rm -f /tmp/disasm_$$.co
echo "$OUT"
