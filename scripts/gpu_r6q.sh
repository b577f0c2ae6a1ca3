#!/bin/bash
# round 6: wave-per-token k-only rope / KV write: numerics, then the round-5 tree vs this tree (microbench small)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
timeout -k 10 600 $PYT --timeout 120 -m gpu tests/test_kernels_gpu.py -k "rope or paged_decode" > gpurun_out/r6q_k.log 2>&1; rc=$?
tail -3 gpurun_out/r6q_k.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  (cd ab_old && timeout -k 10 300 python3 -u scripts/microbench.py small > $ROOT/gpurun_out/r6q_old_$i.log 2>&1) || exit $?
  timeout -k 10 300 python3 -u scripts/microbench.py small > gpurun_out/r6q_new_$i.log 2>&1 || exit $?
done
for f in old_1 new_1 old_2 new_2; do echo "== $f"; grep "rope_kv_write" gpurun_out/r6q_$f.log; done
