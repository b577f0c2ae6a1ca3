#!/bin/bash
# round 6: PMC of gemm4w vs hipBLASLt at config 2's FFN2 shape (HBM-streamed A): bytes fetched, L2 hits
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_enc
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --stats --output-format csv \
  -d gpurun_out/pmc_enc -o run -- python3 scripts/probes/enc_pmc.py > gpurun_out/pmc_enc.log 2>&1
rc=$?; echo "rc=$rc"; find gpurun_out/pmc_enc -name "*.csv" | head; exit $rc
