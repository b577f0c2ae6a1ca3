#!/bin/bash
# PMC counters of gate|up + SwiGLU at the headline decode batch: gemm4w VAR 64 (TR epilogue) vs VAR 96 (staged
# epilogue) vs hipBLASLt; one rocprofv3 run per pass (SQ <= 8, GRBM <= 2 counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$R"
: > gpurun_out/pmc/summary_g4tr.txt
for kind in ${KINDS:-g4v64 g4v96 blas}; do
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc/${kind}_${tag} -o run -- \
      python3 scripts/probes/g4_run.py $kind 10 > gpurun_out/pmc/g4tr_${kind}_${tag}.log 2>&1 || exit 1
    echo "## $kind" >> gpurun_out/pmc/summary_g4tr.txt
    python3 scripts/pmc_summary.py /tmp/pmc/${kind}_${tag} >> gpurun_out/pmc/summary_g4tr.txt 2>&1
  done
done
cat gpurun_out/pmc/summary_g4tr.txt
