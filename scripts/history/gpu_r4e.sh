#!/bin/bash
# Round 4: readfirstlane-uniform buffer resources (no waterfall loops in gemm8g's main loop / the GEMM
# epilogues) — numerics of every GEMM core, the model tests, GEMM + MoE A/Bs, the headline bench
# (unprofiled) and config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "gemm or moe or fp8 or grouped" > gpurun_out/pytest_r4e.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r4e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_tp_gpu.py tests/test_model_gpu.py > gpurun_out/pytest_r4e2.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r4e2.log; [ $rc -eq 0 ] || exit $rc
G4_VARS="32,64" G4_VARS_EPI="32,64" G4_SHAPES="1,3,4" timeout -k 10 400 python3 -u scripts/microbench.py g4ab \
    > gpurun_out/micro_g4_r4e.log 2>&1
rc=$?; echo "g4ab rc=$rc"; grep g4ab gpurun_out/micro_g4_r4e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/moe_gemm_ab.py > gpurun_out/moe_ab_r4e.log 2>&1
rc=$?; echo "moe ab rc=$rc"; tail -8 gpurun_out/moe_ab_r4e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 5 --warmup 2 > gpurun_out/bench_r4e.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_r4e.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
ONLY=moe MOE_R=32 bash scripts/gpu_configs.sh
