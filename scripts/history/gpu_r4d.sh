#!/bin/bash
# Round 4: sampler rewrite (packed u16 threshold masses, fma+exp2 u pass, one-wave walk) and q RoPE at load
# in the decode kernels (rope_kv_write k-only on pure decode steps) — numerics, the dense TP=2 encode test,
# the model/engine tests, the sampler + prefix microbenches, then the EP probe and the bench profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "sample or paged_decode or rope or gemm4w or gemm8p or silu or swiglu" > gpurun_out/pytest_r4d.log 2>&1
rc=$?; echo "pytest kernels rc=$rc"; tail -3 gpurun_out/pytest_r4d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_tp_gpu.py tests/test_model_gpu.py tests/test_bench_rehearsal_gpu.py > gpurun_out/pytest_r4d2.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 gpurun_out/pytest_r4d2.log; [ $rc -eq 0 ] || exit $rc
MICRO_PREFIX_QUICK=1 timeout -k 10 300 python3 -u scripts/microbench.py sample prefix > gpurun_out/micro_r4d.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_r4d.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/microbench.py small > gpurun_out/micro_small_r4d.log 2>&1
rc=$?; echo "micro small rc=$rc"; grep "rope\|silu" gpurun_out/micro_small_r4d.log; [ $rc -eq 0 ] || exit $rc
G4_VARS="32,64" G4_VARS_EPI="32,64" G4_SHAPES="0,1,2,3,4" timeout -k 10 400 python3 -u scripts/microbench.py g4ab \
    > gpurun_out/micro_g4_r4d.log 2>&1
rc=$?; echo "g4ab rc=$rc"; grep g4ab gpurun_out/micro_g4_r4d.log; [ $rc -eq 0 ] || exit $rc
bash scripts/history/gpu_r4c.sh
