#!/bin/bash
# round 6 final: same-box headline A/B of the round-5 final tree (ab_old/) vs this tree, driver command
# shortened to 5 timed steps, ABBA
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for arm in old new new old; do
  i=$((i + 1))
  if [ $arm = old ]; then
    (cd ab_old && timeout -k 10 500 python3 -u bench.py --steps 5 --warmup 2 > $ROOT/gpurun_out/r6y_${arm}_$i.log 2>&1) || exit $?
  else
    timeout -k 10 500 python3 -u bench.py --steps 5 --warmup 2 > gpurun_out/r6y_${arm}_$i.log 2>&1 || exit $?
  fi
  echo "$arm $i: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r6y_${arm}_$i.log | tr '\n' ' ')"
done
