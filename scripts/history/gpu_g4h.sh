#!/bin/bash
# gemm4w library-shaped schedule (LWC_G4_VAR=32): fp32-oracle numerics for both schedules, then the A/B
# against hipBLASLt / gemm8p / the default schedule (scripts/microbench.py g4ab), then the serving A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "gemm4w" > gpurun_out/pytest_g4h.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_g4h.log; [ $rc -eq 0 ] || exit $rc
G4_VARS="1,32" G4_VARS_EPI="1,32" G4_SHAPES="0,1,2,3,4" timeout -k 10 600 python -u scripts/microbench.py g4ab > gpurun_out/micro_g4h.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_g4h.log; [ $rc -eq 0 ] || exit $rc
bash scripts/history/gpu_serve_r4.sh
