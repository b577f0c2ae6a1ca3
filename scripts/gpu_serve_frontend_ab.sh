#!/bin/bash
# Serving A/B of the front end: the tree at ab_old/ (a snapshot of an earlier commit's Python package, run
# with this tree's built .so files) vs this tree, interleaved on one box (old, new, old, new), same load.
# Make the snapshot first (git-ignored):  mkdir ab_old && git archive <commit> llm_weighted_consensus_amd
#   scripts/serve_load.py | tar -x -C ab_old && cp llm_weighted_consensus_amd/ops/_kernels.so ab_old/llm_weighted_consensus_amd/ops/
#   && cp llm_weighted_consensus_amd/_runtime.so ab_old/llm_weighted_consensus_amd/   (round 5 used a34f755)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$(pwd)
for r in 1 2; do
  for arm in old new; do
    if [ $arm = old ]; then dir=$ROOT/ab_old; else dir=$ROOT; fi
    (cd $dir && timeout -k 10 300 python3 -u scripts/serve_load.py --requests ${SERVE_N:-256} --concurrency 64 \
        > $ROOT/gpurun_out/serve_fe_${arm}_$r.log 2>&1)
    rc=$?; echo "run $r $arm rc=$rc"; grep '"metric"' gpurun_out/serve_fe_${arm}_$r.log | cut -c1-400
    [ $rc -eq 0 ] || exit $rc
  done
done
