set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_chunked_prefill_gpu.py tests/test_preemption_gpu.py > gpurun_out/mixed2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/mixed2_tests.log | tail -30
[ $rc -eq 0 ] || { tail -50 gpurun_out/mixed2_tests.log; exit $rc; }
CHUNKS="2048 512" bash scripts/gpu_serve_ab.sh
