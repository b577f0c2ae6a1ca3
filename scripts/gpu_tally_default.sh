#!/bin/bash
# The batched GPU tally on by default with an in-process engine: server GPU tests, then the serving load.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_server_gpu.py tests/test_vote_tally.py -m gpu > gpurun_out/tally_default_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tally_default_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/serve_load.py --requests 256 --concurrency 64 > gpurun_out/serve_default.log 2>&1
rc=$?; echo "serve rc=$rc"; grep '"metric"' gpurun_out/serve_default.log | cut -c1-330
grep -o '"gpu_tally": {[^}]*}' gpurun_out/serve_default.log
exit $rc
