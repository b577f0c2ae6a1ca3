#!/bin/bash
# round 6: serving with the TunableOp table off / on (ABBA), then the headline bench (3 steps) off / on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CMD="python3 -u scripts/serve_load.py --requests 256 --concurrency 64"
i=0
for arm in 0 1 1 0 0 1; do
  i=$((i + 1))
  LWC_TUNED_BLAS=$arm timeout -k 10 400 $CMD > gpurun_out/r6t_serve_${arm}_$i.log 2>&1 || exit $?
  echo "tuned_blas=$arm run $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*' gpurun_out/r6t_serve_${arm}_$i.log | tr '\n' ' ')"
done
for arm in 0 1; do
  LWC_TUNED_BLAS=$arm timeout -k 10 500 python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/r6t_bench_$arm.log 2>&1 || exit $?
  echo "bench tuned_blas=$arm: $(grep -o '"value": [0-9.]*' gpurun_out/r6t_bench_$arm.log)"
done
