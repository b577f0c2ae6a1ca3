#!/bin/bash
# (Round-3 experiment, reverted: profiles/bench_r64_round3.md.)  Persistent sampler with next-row LDS prefetch: sampler tests (incl. prefetch == per-row kernel), then the
# standalone sampler timing: this tree with prefetch on / off and the pre-change tree (_ab_orig), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py -m gpu -k "sample" > gpurun_out/samp_pf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/samp_pf_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  LWC_SAMPLE_PREFETCH=1 timeout -k 10 60 python scripts/sample_probe.py 4096 20 || exit 1
  LWC_SAMPLE_PREFETCH=0 timeout -k 10 60 python scripts/sample_probe.py 4096 20 || exit 1
  # the round-3 A/B also timed a copy of the previous tree here (built under _ab_orig/, since removed)
done
