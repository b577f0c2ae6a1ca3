#!/bin/bash
# Round 3 checkpoint: the whole GPU test suite + smoke, then the headline with the measured GEMM plan vs the
# plan biased to the hand-written cores (LWC_GEMM_OWN_MARGIN=0.10: a hand-written core within 10 % of
# hipBLASLt is taken), back to back on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_r3c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_r3c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3c.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_r3c.log; [ $rc -eq 0 ] || exit $rc
for m in 0.01 0.10 0.01 0.10; do
  LWC_GEMM_OWN_MARGIN=$m timeout -k 10 600 python bench.py --steps 3 --warmup 1 --profile-steps > gpurun_out/bench_m$m.log 2>&1
  rc=$?; echo "margin=$m rc=$rc"; grep "choice=" gpurun_out/bench_m$m.log | grep -v 65536 | sed 's/^/  /'
  tail -1 gpurun_out/bench_m$m.log | cut -c1-170; [ $rc -eq 0 ] || exit $rc
done
