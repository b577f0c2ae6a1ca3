#!/bin/bash
# round 6: gemm4w takes A of any size in one launch (per-tile A resource): numerics, encoder GEMMs, config 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 200 -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py -k "gemm4w or bert" \
  > gpurun_out/r6w_k.log 2>&1; rc=$?
tail -3 gpurun_out/r6w_k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/microbench.py enc > gpurun_out/r6w_enc.log 2>&1 || exit $?
grep "enc M" gpurun_out/r6w_enc.log
for i in 1 2; do
  timeout -k 10 300 python3 -u bench_configs.py encoder --steps 3 > gpurun_out/r6w_cfg2_$i.log 2>&1 || exit $?
  echo "config 2 run $i: $(grep -o '"value": [0-9.]*' gpurun_out/r6w_cfg2_$i.log)"
  grep "enc_residual\|:bias" gpurun_out/r6w_cfg2_$i.log | cut -c1-200
done
