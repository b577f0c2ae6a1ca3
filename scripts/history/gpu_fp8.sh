#!/bin/bash
# Round 3: dense fp8 on the hand-written core (gemm8g dense mode), fused RMSNorm+e4m3, K10b vote tally —
# kernel tests, then config 5 with the library fp8 GEMM vs the planner (A/B in one call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_vote_tally.py tests/test_alltoall_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu \
    -k "tally or fp8 or rmsnorm or gemm8g or alltoall" > gpurun_out/fp8_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/fp8_tests.log; [ $rc -eq 0 ] || exit $rc
LWC_FP8_GEMM=blas timeout -k 10 600 python bench_configs.py moe --requests 32 --steps 2 > gpurun_out/moe_blas.log 2>&1
rc=$?; echo "moe blas rc=$rc"; tail -3 gpurun_out/moe_blas.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench_configs.py moe --requests 32 --steps 2 > gpurun_out/moe_auto.log 2>&1
rc=$?; echo "moe auto rc=$rc"; tail -12 gpurun_out/moe_auto.log
exit $rc
