#!/bin/bash
# round 6: same-box serving A/B of the round-5 final tree (ab_old/) vs this tree, 3 interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64"
for i in 1 2 3; do
  (cd ab_old && timeout -k 10 400 $CMD > $ROOT/gpurun_out/r6i_old_$i.log 2>&1); rc=$?
  echo "old $i rc=$rc: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*' gpurun_out/r6i_old_$i.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 400 $CMD > gpurun_out/r6i_new_$i.log 2>&1; rc=$?
  echo "new $i rc=$rc: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*' gpurun_out/r6i_new_$i.log | tr '\n' ' ')"; [ $rc -ne 0 ] && exit $rc
done
