#!/bin/bash
# gemm4w / gemm8p tile-group size (LWC_G8_GM: m-tiles per group of the tile order) on the o / down / lm_head
# shapes vs hipBLASLt, one process per setting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for gm in 8 4 16 2; do
  LWC_G8_GM=$gm G4_SHAPES=1,3,4 timeout -k 10 300 python -u scripts/microbench.py g4ab > gpurun_out/gm$gm.log 2>&1
  rc=$?; echo "gm=$gm rc=$rc"; grep g4ab gpurun_out/gm$gm.log; [ $rc -eq 0 ] || exit $rc
done
