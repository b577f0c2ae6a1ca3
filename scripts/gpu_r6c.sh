#!/bin/bash
# round 6: split-K numerics, then the stamps probe (per-XCD ends)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 120 -m gpu tests/test_kernels_gpu.py -k "gemm4w" > gpurun_out/r6c_k.log 2>&1; rc=$?
tail -15 gpurun_out/r6c_k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 scripts/probes/g4_stamps > gpurun_out/stamps_r6c.log 2>&1; rc=$?
grep -E "^==|starts|per XCD" gpurun_out/stamps_r6c.log; exit $rc
