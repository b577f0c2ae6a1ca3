#!/bin/bash
# Residual epilogue with branch-free batched residual loads (gemm4w / gemm8p): GEMM tests, the o / down
# shapes A/B vs hipBLASLt (microbench g4ab), the headline bench with its per-shape plan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -k "gemm or residual or decoder" > gpurun_out/res_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/res_tests.log; [ $rc -eq 0 ] || exit $rc
G4_SHAPES=1,3 timeout -k 10 300 python -u scripts/microbench.py g4ab > gpurun_out/res_g4ab.log 2>&1
rc=$?; echo "g4ab rc=$rc"; grep g4ab gpurun_out/res_g4ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --profile-steps > gpurun_out/bench_res.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "choice=" gpurun_out/bench_res.log | grep -v 65536; tail -1 gpurun_out/bench_res.log | cut -c1-170
exit $rc
