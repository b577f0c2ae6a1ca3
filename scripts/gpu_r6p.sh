#!/bin/bash
# round 6: polynomial packed GELU in gemm4w VAR 64: numerics, then the encoder GEMMs of the round-5 tree vs
# this tree (interleaved), then config 2 on this tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 120 -m gpu tests/test_kernels_gpu.py -k "gemm4w or gemm8p_bias" > gpurun_out/r6p_k.log 2>&1; rc=$?
tail -3 gpurun_out/r6p_k.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  (cd ab_old && timeout -k 10 300 python3 -u scripts/microbench.py enc > $ROOT/gpurun_out/r6p_old_$i.log 2>&1) || exit $?
  timeout -k 10 300 python3 -u scripts/microbench.py enc > gpurun_out/r6p_new_$i.log 2>&1 || exit $?
done
for f in old_1 new_1 old_2 new_2; do echo "== $f"; grep "enc M" gpurun_out/r6p_$f.log; done
timeout -k 10 300 python3 -u bench_configs.py encoder --steps 3 > gpurun_out/r6p_cfg2.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/r6p_cfg2.log
