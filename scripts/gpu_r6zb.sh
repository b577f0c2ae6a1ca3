#!/bin/bash
# round 6 final tree: serving load test and config 2, one run each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 -u scripts/serve_load.py --requests 256 --concurrency 64 > gpurun_out/r6zb_serve.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"p99": [0-9.]*' gpurun_out/r6zb_serve.log | tr '\n' ' '; echo
timeout -k 10 300 python3 -u bench_configs.py encoder --steps 3 > gpurun_out/r6zb_cfg2.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/r6zb_cfg2.log
