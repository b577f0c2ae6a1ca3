#!/bin/bash
# Round 4: EP device-exchange tests, cascade decode microbench (prefix pass overlapped with the suffix),
# then the headline bench.  Each GPU step under its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_alltoall_gpu.py tests/test_kernels_gpu.py -k "alltoall or ep_ or ep2 or cascade" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r4a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_r4a.log; [ $rc -eq 0 ] || exit $rc
MICRO_PREFIX_QUICK=1 timeout -k 10 300 python -u scripts/microbench.py prefix > gpurun_out/micro_prefix_r4.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_prefix_r4.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_r4a.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_r4a.log | cut -c1-400
exit $rc
