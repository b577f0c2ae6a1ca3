#!/bin/bash
# Round 4: decode attention with 16 B V loads + K=16 PV MFMAs — every decode-attention / model / engine GPU
# test, the cascade microbench, then the headline bench.  Each GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_chunked_prefill_gpu.py -k "decode or cascade or model or engine or chunked or graph" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r4b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_r4b.log; [ $rc -eq 0 ] || exit $rc
MICRO_PREFIX_QUICK=1 timeout -k 10 300 python -u scripts/microbench.py prefix > gpurun_out/micro_prefix_r4b.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_prefix_r4b.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_r4b.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_r4b.log | cut -c1-300
exit $rc
