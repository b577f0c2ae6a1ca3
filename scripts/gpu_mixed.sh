set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py::test_prefill_attention_paged tests/test_chunked_prefill_gpu.py tests/test_preemption_gpu.py > gpurun_out/mixed_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/mixed_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/prefill_probe.py > gpurun_out/prefill_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/prefill_probe.log | grep -v amdgpu.ids
exit $rc
