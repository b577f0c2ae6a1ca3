#!/bin/bash
# round 6: split-K as a compile-time build (the unsplit kernels back to the round-5 code): gemm4w numerics,
# then serving-shape GEMMs of the round-5 tree vs this tree (interleaved twice)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 120 -m gpu tests/test_kernels_gpu.py -k "gemm4w" > gpurun_out/r6m_k.log 2>&1; rc=$?
tail -3 gpurun_out/r6m_k.log; [ $rc -ne 0 ] && exit $rc
export SERVE_M=1024,2048,2560,3072
for i in 1 2; do
  (cd ab_old && timeout -k 10 300 python3 -u scripts/microbench.py serve > $ROOT/gpurun_out/r6m_old_$i.log 2>&1) || exit $?
  timeout -k 10 300 python3 -u scripts/microbench.py serve > gpurun_out/r6m_new_$i.log 2>&1 || exit $?
done
for f in old_1 new_1 old_2 new_2; do echo "== $f $(grep -E "gu g4p|qkv g4:|o g4:" gpurun_out/r6m_$f.log | awk '{print $2, $3, $5}' | tr '\n' ';')"; done
