#!/bin/bash
# round 6: same-box A/B of the round-5 final tree (ab_old/) vs this tree: headline bench (interleaved, the new
# tree with the coordinate-descent step A/B) and the decode-shape GEMM microbench of both trees
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  (cd ab_old && timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 > $ROOT/gpurun_out/r6b_old_$i.log 2>&1); rc=$?
  echo "old $i rc=$rc: $(grep -o '"value": [0-9.]*' gpurun_out/r6b_old_$i.log)"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 > gpurun_out/r6b_new_$i.log 2>&1; rc=$?
  echo "new $i rc=$rc: $(grep -o '"value": [0-9.]*' gpurun_out/r6b_new_$i.log)"; grep "step A/B" gpurun_out/r6b_new_$i.log | cut -c1-1500
  [ $rc -ne 0 ] && exit $rc
done
(cd ab_old && G4_SHAPES=1,2,3,4 G4_VARS=64 G4_VARS_EPI=64 timeout -k 10 600 python3 scripts/microbench.py g4ab > $ROOT/gpurun_out/g4ab_old.log 2>&1); rc=$?
cut -c1-300 gpurun_out/g4ab_old.log; [ $rc -ne 0 ] && exit $rc
G4_SHAPES=1,2,3,4 G4_VARS=64 G4_NO_G8=1 timeout -k 10 600 python3 scripts/microbench.py g4ab > gpurun_out/g4ab_new.log 2>&1; rc=$?
cut -c1-300 gpurun_out/g4ab_new.log; exit $rc
