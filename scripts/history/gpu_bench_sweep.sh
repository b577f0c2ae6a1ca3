#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for R in ${SWEEP_R:-4 8 16}; do
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 --requests $R --profile-steps > gpurun_out/bench_r$R.log 2>&1
  rc=$?; echo "R=$R rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_r$R.log | tail -3
  [ $rc -eq 0 ] || exit $rc
done
