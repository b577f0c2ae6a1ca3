#!/bin/bash
# Round 4: dense MX MLP (embedder prefill) — numerics, TP / model tests, config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "mx or fp8 or gemm8g" > gpurun_out/pytest_r4o.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r4o.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_tp_gpu.py tests/test_model_gpu.py > gpurun_out/pytest_r4o2.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r4o2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench_configs.py moe --steps 2 > gpurun_out/cfg5_r4o.log 2> gpurun_out/cfg5_r4o.err
rc=$?; echo "config5 rc=$rc"; tail -1 gpurun_out/cfg5_r4o.log | cut -c1-200; exit $rc
