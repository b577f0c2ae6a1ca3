#!/bin/bash
# round 6: serving-shape GEMMs, round-5 tree vs this tree on one box (interleaved twice)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export SERVE_M=1024,2048,2304,2560,3072
for i in 1 2; do
  (cd ab_old && timeout -k 10 300 python3 -u scripts/microbench.py serve > $ROOT/gpurun_out/r6l_old_$i.log 2>&1) || exit $?
  timeout -k 10 300 python3 -u scripts/microbench.py serve > gpurun_out/r6l_new_$i.log 2>&1 || exit $?
done
for f in old_1 new_1 old_2 new_2; do echo "== $f"; grep -E "gu |o g4:|down g4:|qkv g4:" gpurun_out/r6l_$f.log | grep -v g4s | tr '\n' ';' | cut -c1-2000; echo; done
