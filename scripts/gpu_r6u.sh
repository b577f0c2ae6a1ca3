#!/bin/bash
# round 6: engine pinned upload ring + TunableOp off by default: engine / model GPU tests, then serving ABBA
# against the round-5 tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 900 $PYT --timeout 200 -m gpu tests/test_model_gpu.py tests/test_chunked_prefill_gpu.py tests/test_preemption_gpu.py \
  > gpurun_out/r6u_k.log 2>&1; rc=$?
tail -3 gpurun_out/r6u_k.log; [ $rc -ne 0 ] && exit $rc
CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64"
i=0
for arm in old new new old old new; do
  i=$((i + 1))
  if [ $arm = old ]; then
    (cd ab_old && timeout -k 10 400 $CMD > $ROOT/gpurun_out/r6u_${arm}_$i.log 2>&1) || exit $?
  else
    timeout -k 10 400 $CMD > gpurun_out/r6u_${arm}_$i.log 2>&1 || exit $?
  fi
  echo "$arm $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*\|"decode.process": [^]]*' gpurun_out/r6u_${arm}_$i.log | tr '\n' ' ')"
done
