#!/bin/bash
# Round 4: config 5 (64 requests) after the gemm8g slot-major order + empty-block MFMA skip.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python3 bench_configs.py moe --steps 2 > gpurun_out/cfg5_r4m.log 2> gpurun_out/cfg5_r4m.err
rc=$?; echo "config5 rc=$rc"; tail -1 gpurun_out/cfg5_r4m.log | cut -c1-200; exit $rc
