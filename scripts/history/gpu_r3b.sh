#!/bin/bash
# Round 3: dense fp8 (grouped tile order) and encoder GEMM planner with gemm4w — kernel tests, config 5,
# config 2, the headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -k "fp8 or gemm8g or gemm4w or bert or encoder" \
    > gpurun_out/r3b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r3b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench_configs.py moe --requests 32 --steps 2 > gpurun_out/moe_auto2.log 2>&1
rc=$?; echo "moe rc=$rc"; grep -v amdgpu.ids gpurun_out/moe_auto2.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_configs.py encoder > gpurun_out/enc.log 2>&1
rc=$?; echo "encoder rc=$rc"; grep -v amdgpu.ids gpurun_out/enc.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_r3b.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_r3b.log
exit $rc
