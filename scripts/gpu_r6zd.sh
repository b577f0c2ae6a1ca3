#!/bin/bash
# round 6: paired-ratio move races in the in-step A/B: its GPU test, then the driver's bench command twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "graph_equivalence" > gpurun_out/r6zd_test.log 2>&1 || { tail -30 gpurun_out/r6zd_test.log; exit 1; }
tail -1 gpurun_out/r6zd_test.log
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6zd_bench_$i.log 2>&1 \
    || { tail -30 gpurun_out/r6zd_bench_$i.log; exit 1; }
  grep '"metric"' gpurun_out/r6zd_bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['decode_plan'], d['step_ab_ms'])"
done
