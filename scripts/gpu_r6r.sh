#!/bin/bash
# round 6: split-K of the experts' ragged last tiles in gemm8g: numerics, the routed-expert microbench with the
# split off / 2 / 4 (interleaved), then config 5 with the split off / on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 120 -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py -k "gemm8g or grouped or moe or mixtral" \
  > gpurun_out/r6r_k.log 2>&1; rc=$?
tail -3 gpurun_out/r6r_k.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for sp in 1 4; do
    LWC_G8G_SPLIT=$sp MICRO_MOE_T=4096 timeout -k 10 300 python3 -u scripts/microbench.py moe > gpurun_out/r6r_moe_${sp}_$i.log 2>&1 || exit $?
    echo "split $sp run $i: $(grep 'moe fp8' gpurun_out/r6r_moe_${sp}_$i.log | tr '\n' ' ' | cut -c1-400)"
  done
done
for sp in 1 4; do
  LWC_G8G_SPLIT=$sp timeout -k 10 600 python3 -u bench_configs.py moe --steps 2 > gpurun_out/r6r_cfg5_$sp.log 2>&1 || exit $?
  echo "config 5 split $sp: $(grep -o '"value": [0-9.]*' gpurun_out/r6r_cfg5_$sp.log)"
done
