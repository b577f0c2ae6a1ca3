#!/bin/bash
# round 6: serving A/B (mixed-step buckets: gate|up only vs every projection, split-K available), then the
# serving rocprof
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_ROUNDS=2 AB_CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64" \
  bash scripts/gpu_ab.sh "LWC_GEMM_BUCKETS=swiglu" "LWC_GEMM_BUCKETS=1" || exit $?
grep -h "gemm_plan\|score requests" gpurun_out/ab_2_r2.log | cut -c1-600
bash scripts/gpu_profile_serve.sh
