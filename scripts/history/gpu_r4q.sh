#!/bin/bash
# Round 4: moe_route with per-wave aggregated counters — route test, MoE / EP tests, config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "route or moe or grouped or mx" > gpurun_out/pytest_r4q.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r4q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_model_gpu.py tests/test_tp_gpu.py tests/test_alltoall_gpu.py -k "mixtral or moe or ep" > gpurun_out/pytest_r4q2.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r4q2.log; [ $rc -eq 0 ] || exit $rc
MOE_R=64 bash scripts/gpu_profile_moe.sh > gpurun_out/prof_r4q.log 2>&1
rc=$?; echo "profile rc=$rc"; grep "moe_route\|moe_combine" gpurun_out/prof_moe_summary.md | cut -c1-160; tail -1 gpurun_out/prof_moe.log | cut -c1-160
exit $rc
