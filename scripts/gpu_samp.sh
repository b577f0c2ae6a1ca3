set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sample" > gpurun_out/samp_tests.log 2>&1
rc=$?; echo "sampler tests rc=$rc"; tail -3 gpurun_out/samp_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/samp_tests.log | head; exit $rc; }
timeout -k 10 300 python -u scripts/microbench.py sample > gpurun_out/samp_micro.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/samp_micro.log; exit $rc
