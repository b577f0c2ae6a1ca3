#!/bin/bash
# BASELINE configs 2, 3 and 5 (TP=1) on one MI355X; results -> gpurun_out/configs.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
: > gpurun_out/configs.log
if [ "${ONLY:-}" != "moe" ] && [ "${ONLY:-}" != "tp2" ]; then
timeout -k 10 240 python bench_configs.py encoder >> gpurun_out/configs.log 2> gpurun_out/configs_err.log
rc=$?; echo "config2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --candidates 32 --steps 2 --warmup 1 >> gpurun_out/configs.log 2>> gpurun_out/configs_err.log
rc=$?; echo "config3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
[ "${ONLY:-}" = "small" ] && { cat gpurun_out/configs.log; exit 0; }
rc=0
if [ "${ONLY:-}" != "tp2" ]; then
  timeout -k 10 1000 python bench_configs.py moe --requests ${MOE_R:-64} --steps 2 >> gpurun_out/configs.log 2>> gpurun_out/configs_err.log
  rc=$?; echo "config5 rc=$rc"
fi
if [ $rc -eq 0 ] && [ -n "${TP2:-}" ]; then
  # TP=2 through the IPC all-reduce; on a one-GPU box both ranks share the GPU (protocol rehearsal)
  # (TP2_GPUS=4: two TP=2 groups, data-parallel across them, each group its own all-reduce)
  LWC_SHARE_ONE_GPU=${SHARE:-1} timeout -k 10 1000 python bench_configs.py moe --tp 2 --gpus ${TP2_GPUS:-2} \
      --requests ${TP2_R:-16} --steps 2 --tp-comm ${TP2_COMM:-ipc} \
      >> gpurun_out/configs.log 2>> gpurun_out/configs_err.log
  rc=$?; echo "config5 tp2 rc=$rc"
fi
cat gpurun_out/configs.log
exit $rc
