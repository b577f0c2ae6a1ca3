#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python scripts/microbench.py ${MICRO_WHAT:-gemm attn sample small} > gpurun_out/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/micro.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
if [ -n "$TUNE" ]; then
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop.csv \
    timeout -k 10 900 python scripts/microbench.py gemm > gpurun_out/micro_tuned.log 2>&1
  rc=$?; echo "tuned rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_tuned.log
fi
exit $rc
