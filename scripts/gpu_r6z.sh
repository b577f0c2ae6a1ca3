#!/bin/bash
# round 6: mixed-step buckets for every projection (two-point bucket timing, TunableOp off) vs gate|up only, ABBA
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64"
i=0
for arm in swiglu 1 1 swiglu swiglu 1; do
  i=$((i + 1))
  LWC_GEMM_BUCKETS=$arm timeout -k 10 400 $CMD > gpurun_out/r6z_${arm}_$i.log 2>&1 || exit $?
  echo "$arm $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*' gpurun_out/r6z_${arm}_$i.log | tr '\n' ' ')"
done
