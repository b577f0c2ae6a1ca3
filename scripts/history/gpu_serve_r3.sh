#!/bin/bash
# Serving on the round-3 tree: chunk 2048 (default) and 4096, and chunk 2048 with the batched GPU tally
# (LWC_GPU_TALLY=2), one JSON line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CHUNKS="2048 4096" bash scripts/gpu_serve_ab.sh || exit $?
LWC_GPU_TALLY=2 LWC_CHUNKED_PREFILL=2048 timeout -k 10 300 python3 -u scripts/serve_load.py --requests 256 \
    --concurrency 64 > gpurun_out/serve_tally.log 2>&1
rc=$?; echo "tally rc=$rc"; grep '"metric"' gpurun_out/serve_tally.log | cut -c1-420
grep -o '"gpu_tally": {[^}]*}' gpurun_out/serve_tally.log
exit $rc
