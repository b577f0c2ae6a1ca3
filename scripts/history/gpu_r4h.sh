#!/bin/bash
# Round 4: SwiGLU in gemm8g's epilogue for the fp8 MoE experts — numerics (kernel + Mixtral model / TP / EP
# tests), the MoE-middle A/B, config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "gemm8g or grouped or moe or fp8" > gpurun_out/pytest_r4h.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r4h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_tp_gpu.py tests/test_model_gpu.py tests/test_alltoall_gpu.py > gpurun_out/pytest_r4h2.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r4h2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/moe_swiglu_ab.py > gpurun_out/moe_swiglu_r4h.log 2>&1
rc=$?; echo "ab rc=$rc"; grep "T=" gpurun_out/moe_swiglu_r4h.log; [ $rc -eq 0 ] || exit $rc
for R in 32 64; do
  timeout -k 10 900 python3 bench_configs.py moe --requests $R --steps 2 > gpurun_out/cfg5_r4h_r$R.log 2> gpurun_out/cfg5_r4h_r$R.err
  rc=$?; echo "config5 R=$R rc=$rc"; tail -1 gpurun_out/cfg5_r4h_r$R.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
