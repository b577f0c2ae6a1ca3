#!/bin/bash
# Round 4: greedy sampler rewrite (numerics + microbench), then a rocprofv3 profile of the serving load.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "sample" > gpurun_out/pytest_r4f.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r4f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/microbench.py sample > gpurun_out/micro_sample_r4f.log 2>&1
rc=$?; echo "micro rc=$rc"; grep "B=4096" gpurun_out/micro_sample_r4f.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profile_serve.sh
