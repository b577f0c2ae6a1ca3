#!/bin/bash
# round 6: stride probe, gemm4w tile-order group sizes on the decode shapes, quick bench with the step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 scripts/probes/stride_probe.py > gpurun_out/stride.log 2>&1; rc=$?
cat gpurun_out/stride.log; [ $rc -ne 0 ] && exit $rc
G4_SHAPES=1,2,3,4 G4_VARS=64 G4_GMS=4,8,16 G4_NO_G8=1 timeout -k 10 600 python3 scripts/microbench.py g4ab > gpurun_out/g4ab_gm.log 2>&1; rc=$?
cat gpurun_out/g4ab_gm.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py --steps 2 --warmup 1 > gpurun_out/r6a_bench.log 2>&1; rc=$?
grep -v "^# warmup\|^# timed" gpurun_out/r6a_bench.log | tail -6; exit $rc
