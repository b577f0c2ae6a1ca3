set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "decode" > gpurun_out/dec_tests.log 2>&1
rc=$?; echo "decode tests rc=$rc"; tail -3 gpurun_out/dec_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/microbench.py attn > gpurun_out/dec_micro.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/dec_micro.log; exit $rc
