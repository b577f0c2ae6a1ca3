#!/bin/bash
# round 6: encoder FFN2-only residual fusion vs none (config 2 A/B), serving with the small-bucket tuning cuts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 120 -m gpu tests/test_model_gpu.py -k "bert" > gpurun_out/r6h_k.log 2>&1; rc=$?
tail -3 gpurun_out/r6h_k.log; [ $rc -ne 0 ] && exit $rc
AB_ROUNDS=2 AB_CMD="python3 -u bench_configs.py encoder --steps 3" \
  bash scripts/gpu_ab.sh "LWC_ENC_FUSED_RESIDUAL=ffn2" "LWC_ENC_FUSED_RESIDUAL=0" || exit $?
AB_ROUNDS=2 AB_CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64" \
  bash scripts/gpu_ab.sh "LWC_GEMM_BUCKETS=swiglu" || exit $?
grep -ho '"phases": {[^}]*}' gpurun_out/ab_1_r1.log gpurun_out/ab_1_r2.log
