#!/bin/bash
# Serving on the round-4 tree (64 concurrent /score/completions, 8 local Llama-3-8B voters each, json_schema):
# interleaved A/B of the host tally (default) vs the batched GPU tally (LWC_GPU_TALLY=2), two runs each on one
# box, one JSON line per run.  Each run under its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for arm in host gpu host gpu; do
  if [ "$arm" = gpu ]; then export LWC_GPU_TALLY=2; else unset LWC_GPU_TALLY; fi
  timeout -k 10 300 python3 -u scripts/serve_load.py --requests 256 --concurrency 64 > gpurun_out/serve_r4_$arm.log 2>&1
  rc=$?; echo "$arm rc=$rc"; grep '"metric"' gpurun_out/serve_r4_$arm.log | cut -c1-400
  grep -o '"gpu_tally": {[^}]*}' gpurun_out/serve_r4_$arm.log
  cat gpurun_out/serve_r4_$arm.log >> gpurun_out/serve_r4_all.log
  [ $rc -eq 0 ] || exit $rc
done
