#!/bin/bash
# End-of-round check on the final tree: the whole GPU suite, smoke, the driver's bench command, and a
# rocprofv3 kernel-trace + stats profile of a short bench run (summary -> gpurun_out/prof_summary.md).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_final_r4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_final_r4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final_r4.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_final_r4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_final_r4.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_final_r4.log | cut -c1-240; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profile.sh
