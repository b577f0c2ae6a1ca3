#!/bin/bash
# GPU validation run used with gpurun: kernel/model tests, smoke, short bench.  Each GPU step has its
# own time limit and the chain stops at the first failure (no GPU step after a fault or timeout).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STAGE=${1:-all}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
[ "$STAGE" = "tests" ] && exit 0
timeout -k 10 900 python bench.py --steps 3 --warmup 1 --profile-steps > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -20 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH_EXTRA" ]; then  # optional A/B variant, e.g. BENCH_EXTRA=--no-prefix-sharing
  timeout -k 10 900 python bench.py --steps 3 --warmup 1 --profile-steps $BENCH_EXTRA > gpurun_out/bench_b.log 2>&1
  rc=$?; echo "bench($BENCH_EXTRA) rc=$rc"; tail -20 gpurun_out/bench_b.log
fi
exit $rc
