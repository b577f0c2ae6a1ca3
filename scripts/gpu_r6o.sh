#!/bin/bash
# round 6 final-tree profiles: headline (bench.py --steps 2), serving load test, config 2 encoder
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 120 -m gpu tests/test_kernels_gpu.py -k "gemm4w" > gpurun_out/r6o_k.log 2>&1; rc=$?
tail -2 gpurun_out/r6o_k.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_profile.sh || exit $?
grep -o '"value": [0-9.]*\|"decode_plan": {[^}]*}' gpurun_out/prof_bench.log
bash scripts/gpu_profile_serve.sh || exit $?
bash scripts/gpu_prof_encoder.sh || exit $?
