#!/bin/bash
# Round 4: gemm8g grouped tile-order A/B (LWC_G8G_GN) at config 5's routed shapes; grouped GEMM tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "gemm8g or grouped or moe" > gpurun_out/pytest_r4l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4l.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/g8g_order_ab.py > gpurun_out/g8g_order_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/g8g_order_ab.log | tail -6; exit $rc
