set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "knn" > gpurun_out/knn.log 2>&1
rc=$?; echo "knn rc=$rc"; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/knn.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/microbench.py bw sample > gpurun_out/micro_bw2.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/micro_bw2.log; exit $rc
