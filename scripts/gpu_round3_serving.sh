set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tp_serving_gpu.py tests/test_sharded_gpu.py tests/test_chunked_prefill_gpu.py > gpurun_out/serving_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/serving_tests.log | tail -20
[ $rc -eq 0 ] || { tail -60 gpurun_out/serving_tests.log; exit $rc; }
bash scripts/gpu_serve_ab.sh
