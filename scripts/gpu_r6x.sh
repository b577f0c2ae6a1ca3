#!/bin/bash
# round 6: VAR 65 (VAR 64 with the DMA pieces at the front of seg B) on the encoder shapes and the decode shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 -u scripts/microbench.py enc > gpurun_out/r6x_enc.log 2>&1 || exit $?
grep "enc M" gpurun_out/r6x_enc.log
G4_SHAPES=1,2,3,4 G4_VARS=64,65 G4_NO_G8=1 timeout -k 10 600 python3 -u scripts/microbench.py g4ab > gpurun_out/r6x_g4ab.log 2>&1 || exit $?
grep g4ab gpurun_out/r6x_g4ab.log | cut -c1-300
