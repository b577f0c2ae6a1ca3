#!/bin/bash
# round 6: serving same-box A/B (round-5 tree vs this tree, 3 rounds), the serving rocprof, the driver's bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64"
for i in 1 2 3; do
  (cd ab_old && timeout -k 10 400 $CMD > $ROOT/gpurun_out/r6k_old_$i.log 2>&1) || exit $?
  echo "old $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*' gpurun_out/r6k_old_$i.log | tr '\n' ' ')"
  timeout -k 10 400 $CMD > gpurun_out/r6k_new_$i.log 2>&1 || exit $?
  echo "new $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*' gpurun_out/r6k_new_$i.log | tr '\n' ' ')"
done
bash scripts/gpu_profile_serve.sh || exit $?
timeout -k 10 800 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6k_bench.log 2> gpurun_out/r6k_bench.err
rc=$?; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"decode_plan": {[^}]*}' gpurun_out/r6k_bench.log; exit $rc
