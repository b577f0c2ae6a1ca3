#!/bin/bash
# round 6: split-K with write-through (sc1) partial hand-off: numerics, then the serving-shape microbench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 120 -m gpu tests/test_kernels_gpu.py -k "split" > gpurun_out/r6e_k.log 2>&1; rc=$?
tail -5 gpurun_out/r6e_k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/microbench.py serve > gpurun_out/r6e_serve_mb.log 2>&1; rc=$?
grep -E "o |down |g4s" gpurun_out/r6e_serve_mb.log; exit $rc
