#!/bin/bash
# round 6: encoder residual fused into o / FFN2 + wave LayerNorm: numerics, config-2 A/B (fused, unfused x2),
# then the serving A/B again with the step A/B limited to large buckets, then the encoder profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 120 -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py -k "layernorm or bert or greedy_graph" \
  > gpurun_out/r6g_k.log 2>&1; rc=$?
tail -5 gpurun_out/r6g_k.log; [ $rc -ne 0 ] && exit $rc
AB_ROUNDS=2 AB_CMD="python3 -u bench_configs.py encoder --steps 3" \
  bash scripts/gpu_ab.sh "LWC_ENC_FUSED_RESIDUAL=1" "LWC_ENC_FUSED_RESIDUAL=0" || exit $?
grep -h "gemm_plan\|enc_residual" gpurun_out/ab_1_r2.log | cut -c1-800
AB_ROUNDS=2 AB_CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64" \
  bash scripts/gpu_ab.sh "LWC_GEMM_BUCKETS=swiglu" || exit $?
grep -ho '"phases": {[^}]*}' gpurun_out/ab_1_r1.log gpurun_out/ab_1_r2.log
bash scripts/gpu_prof_encoder.sh
