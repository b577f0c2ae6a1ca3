#!/bin/bash
# gemm4w numerics (fp32 oracle) then the hipBLASLt / gemm8p / gemm4w A/B (scripts/microbench.py g4ab).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LWC_G4_VAR=8 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm4w and plain" -x -q -p no:cacheprovider > gpurun_out/pytest_g4v8.log 2>&1 && echo "v8 tests ok" && timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "${G4_TESTS:-gemm4w}" > gpurun_out/pytest_g4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_g4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/microbench.py g4ab > gpurun_out/micro_g4.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_g4.log
exit $rc
