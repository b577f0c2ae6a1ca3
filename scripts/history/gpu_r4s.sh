#!/bin/bash
# Round 4: decode attention -> MX o-projection operand — kernel + model / TP / EP tests, config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "cascade or mx or fp8 or decode" > gpurun_out/pytest_r4s.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r4s.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_model_gpu.py tests/test_tp_gpu.py tests/test_alltoall_gpu.py tests/test_allreduce_gpu.py \
    tests/test_tp_serving_gpu.py > gpurun_out/pytest_r4s2.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r4s2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench_configs.py moe --steps 2 > gpurun_out/cfg5_r4s.log 2> gpurun_out/cfg5_r4s.err
rc=$?; echo "config5 rc=$rc"; tail -1 gpurun_out/cfg5_r4s.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
LWC_ATTN_MX=0 timeout -k 10 900 python3 bench_configs.py moe --steps 2 > gpurun_out/cfg5_r4s_off.log 2> gpurun_out/cfg5_r4s_off.err
rc=$?; echo "config5 (attn MX off) rc=$rc"; tail -1 gpurun_out/cfg5_r4s_off.log | cut -c1-200; exit $rc
