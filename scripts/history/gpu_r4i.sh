#!/bin/bash
# Round 4: config 5 request sweep above the new default (64), then a kernel profile at 64 requests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for R in 96 128; do
  timeout -k 10 900 python3 bench_configs.py moe --requests $R --steps 2 > gpurun_out/cfg5_r4i_r$R.log 2> gpurun_out/cfg5_r4i_r$R.err
  rc=$?; echo "config5 R=$R rc=$rc"; tail -1 gpurun_out/cfg5_r4i_r$R.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
MOE_R=64 bash scripts/gpu_profile_moe.sh
