#!/bin/bash
# full verification of the tree on one GPU: the GPU test suite, smoke(), the driver's bench command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/suite.log 2>&1 || { tail -30 gpurun_out/suite.log; exit 1; }
tail -2 gpurun_out/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1 \
  || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 \
  || { tail -30 gpurun_out/bench.log; exit 1; }
grep '"metric"' gpurun_out/bench.log
