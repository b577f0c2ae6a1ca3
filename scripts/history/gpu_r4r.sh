#!/bin/bash
# Round 4: moe_route timing check (routing test + a short profile of config 5's decode kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "route" > gpurun_out/pytest_r4r.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r4r.log; [ $rc -eq 0 ] || exit $rc
MOE_R=64 bash scripts/gpu_profile_moe.sh > gpurun_out/prof_r4r.log 2>&1
rc=$?; echo "profile rc=$rc"; grep "moe_route\|moe_combine" gpurun_out/prof_moe_summary.md | cut -c1-160; exit $rc
