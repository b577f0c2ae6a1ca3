set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill_attention or knn or encoder" > gpurun_out/pf2_tests.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/pf2_tests.log | tail -25; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_chunked_prefill_gpu.py tests/test_model_gpu.py > gpurun_out/pf2_model.log 2>&1
rc=$?; echo "model tests rc=$rc"; tail -3 gpurun_out/pf2_model.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/microbench.py pfattn > gpurun_out/pf2_micro.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/pf2_micro.log; exit $rc
