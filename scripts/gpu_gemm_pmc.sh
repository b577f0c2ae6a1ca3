#!/bin/bash
# PMC counters of gemm8p vs hipBLASLt on one shape (run via gpurun).  Each rocprofv3 run is a separate
# process with its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHAPE=${SHAPE:-"4096 4096 4096"}
rocprofv3 -L 2>&1 | grep -oE "(SQ|TCC|TCP|GRBM|TA|TD)_[A-Za-z0-9_]+" | sort -u > gpurun_out/pmc/counters.txt || true
for kind in g8 blas; do
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc/${kind}_${tag} -o run -- \
      python3 scripts/gemm_probe.py $kind $SHAPE 10 > gpurun_out/pmc/${kind}_${tag}.log 2>&1 || exit 1
    python3 scripts/pmc_summary.py /tmp/pmc/${kind}_${tag} >> gpurun_out/pmc/summary.txt 2>&1
  done
done
