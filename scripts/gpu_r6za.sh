#!/bin/bash
# round 6: uneven split-K (S not dividing the K tile count, several rounds of units): tests, then the serving
# mid-size shapes with forced whole-call splits
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -m gpu -k "split_k" > gpurun_out/r6za_tests.log 2>&1 || { tail -30 gpurun_out/r6za_tests.log; exit 1; }
tail -2 gpurun_out/r6za_tests.log
SERVE_M=2304,2560,3072 SERVE_SPLITS=2,3,4,5,6,8 SERVE_ONLY="o ,down ,qkv " timeout -k 10 600 \
  python -u scripts/microbench.py serve > gpurun_out/r6za_serve.log 2>&1 || { tail -30 gpurun_out/r6za_serve.log; exit 1; }
grep "serve M=" gpurun_out/r6za_serve.log
