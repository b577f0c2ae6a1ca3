#!/bin/bash
# round 6: what costs the serving path 6 % against the round-5 tree?  Interleaved on one box: round-5 tree, this
# tree, this tree without split-K in the planner, this tree with the round-5 planner margin
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64"
for i in 1 2; do
  (cd ab_old && timeout -k 10 400 $CMD > $ROOT/gpurun_out/r6j_old_$i.log 2>&1) || exit $?
  echo "old $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*' gpurun_out/r6j_old_$i.log | tr '\n' ' ')"
  timeout -k 10 400 $CMD > gpurun_out/r6j_new_$i.log 2>&1 || exit $?
  echo "new $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*' gpurun_out/r6j_new_$i.log | tr '\n' ' ')"
  LWC_GEMM_NO=g4s timeout -k 10 400 $CMD > gpurun_out/r6j_nos_$i.log 2>&1 || exit $?
  echo "no g4s $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*' gpurun_out/r6j_nos_$i.log | tr '\n' ' ')"


done
