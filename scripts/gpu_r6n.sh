#!/bin/bash
# round 6: same-box serving A/B, round-5 tree vs this tree, ABBA order (old new new old old new new old)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64"
i=0
for arm in old new new old old new new old; do
  i=$((i + 1))
  if [ $arm = old ]; then
    (cd ab_old && timeout -k 10 400 $CMD > $ROOT/gpurun_out/r6n_${arm}_$i.log 2>&1) || exit $?
  else
    timeout -k 10 400 $CMD > gpurun_out/r6n_${arm}_$i.log 2>&1 || exit $?
  fi
  echo "$arm $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*' gpurun_out/r6n_${arm}_$i.log | tr '\n' ' ')"
done
