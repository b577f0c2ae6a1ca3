#!/bin/bash
# Cascade decode: prefix-chunk prefetch (LWC_CASCADE_PREFETCH=1, default) vs the phase order of round 2 —
# cascade tests, microbench A/B (R = 48 / 64, gen 64), then the headline bench with the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py -m gpu -k "cascade or decode" > gpurun_out/casc_pf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/casc_pf_tests.log; [ $rc -eq 0 ] || exit $rc
for pf in 0 1 0 1; do
  LWC_CASCADE_PREFETCH=$pf MICRO_PREFIX_QUICK=1 timeout -k 10 200 python -u scripts/microbench.py prefix \
      > gpurun_out/casc_pf$pf.log 2>&1
  rc=$?; echo "prefetch=$pf rc=$rc"; grep -E "cascade-decode|parts" gpurun_out/casc_pf$pf.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_pf.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_pf.log | cut -c1-200
exit $rc
