#!/bin/bash
# Round 4: last-layer row selection in prefill / the decoder embedder — model, engine, serving GPU tests and
# config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_model_gpu.py tests/test_tp_gpu.py tests/test_chunked_prefill_gpu.py tests/test_preemption_gpu.py \
    tests/test_server_gpu.py tests/test_tp_serving_gpu.py tests/test_alltoall_gpu.py tests/test_allreduce_gpu.py \
    > gpurun_out/pytest_r4p.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4p.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench_configs.py moe --steps 2 > gpurun_out/cfg5_r4p.log 2> gpurun_out/cfg5_r4p.err
rc=$?; echo "config5 rc=$rc"; tail -1 gpurun_out/cfg5_r4p.log | cut -c1-200; exit $rc
