#!/bin/bash
# round 6: serving chunked-prefill budget (rows of prompt per mixed step), interleaved arms (ARMS overrides)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for arm in ${ARMS:-2048 1536 3072 3072 1536 2048}; do
  i=$((i + 1))
  LWC_CHUNKED_PREFILL=$arm timeout -k 10 400 python3 -u scripts/serve_load.py --requests 256 --concurrency 64 \
    > gpurun_out/r6zc_${arm}_$i.log 2>&1 || exit $?
  echo "$arm $i: $(grep -o '"value": [0-9.]*\|"p99": [0-9.]*\|"prefill.mixed": [^]]*' gpurun_out/r6zc_${arm}_$i.log | tr '\n' ' ')"
done
