set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tp_serving_gpu.py > gpurun_out/tp_serve.log 2>&1
rc=$?; echo "rc=$rc"; tail -40 gpurun_out/tp_serve.log; exit $rc
