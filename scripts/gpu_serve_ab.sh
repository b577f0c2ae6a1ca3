#!/bin/bash
# serve_load.py with chunked prefill off / on (mixed decode + chunk forward), one JSON line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in ${CHUNKS:-0 2048 4096}; do
  LWC_CHUNKED_PREFILL=$c timeout -k 10 300 python3 -u scripts/serve_load.py --requests ${SERVE_N:-256} --concurrency 64 \
      > gpurun_out/serve_c$c.log 2>&1
  rc=$?; echo "chunk=$c rc=$rc"; grep '"metric"' gpurun_out/serve_c$c.log | cut -c1-420
  [ $rc -eq 0 ] || exit $rc
done
