#!/bin/bash
# round 6: serving-shape microbench with the split-K arms, then the driver's bench command (step A/B on stderr)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u scripts/microbench.py serve > gpurun_out/r6d_serve_mb.log 2>&1 || exit $?
timeout -k 10 800 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6d_bench.log 2> gpurun_out/r6d_bench.err
rc=$?; tail -3 gpurun_out/r6d_bench.log; grep -iE "step a/b|plan" gpurun_out/r6d_bench.err | tail -30; exit $rc
