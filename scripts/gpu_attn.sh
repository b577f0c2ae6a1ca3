#!/bin/bash
# Decode-attention iteration loop: kernel tests for both decode paths + the attention microbenches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider -k "decode" > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/microbench.py ${MICRO_WHAT:-prefix attn} > gpurun_out/micro_attn.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_attn.log
exit $rc
