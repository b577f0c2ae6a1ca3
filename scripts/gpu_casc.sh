set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_chunked_prefill_gpu.py tests/test_preemption_gpu.py tests/test_model_gpu.py tests/test_server_gpu.py > gpurun_out/casc_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/casc_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/casc_tests.log | head -20; exit $rc; }
CHUNKS="2048" bash scripts/gpu_serve_ab.sh
