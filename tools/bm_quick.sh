#!/bin/bash
# BM match kernel check on the GPU: the BM parity tests, then timings of the
# disparities-on-lanes kernel (auto tile height and a sweep) against the
# 16x16-tile kernel on configs 1 and 2 at batch 1 and 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/bmq
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bm or BM" > gpurun_out/bmq/t.log 2>&1
rc=$?; tail -15 gpurun_out/bmq/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bm_time.py > gpurun_out/bmq/b.txt 2>&1
rc=$?; cat gpurun_out/bmq/b.txt; exit $rc
