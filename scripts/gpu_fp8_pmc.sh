#!/bin/bash
# PMC counters of the dense fp8 GEMMs (gemm4w8 vs gemm8g vs hipBLASLt) on one shape; one rocprofv3 run per pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$R"
SHAPE=${SHAPE:-"16384 6144 4096"}
: > gpurun_out/pmc/summary_fp8.txt
for kind in ${KINDS:-g48 g8g blas}; do
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc/${kind}_${tag} -o run -- \
      python3 scripts/probes/fp8_gemm_run.py $kind $SHAPE 10 > gpurun_out/pmc/fp8_${kind}_${tag}.log 2>&1 || exit 1
    echo "## $kind" >> gpurun_out/pmc/summary_fp8.txt
    python3 scripts/pmc_summary.py /tmp/pmc/${kind}_${tag} >> gpurun_out/pmc/summary_fp8.txt 2>&1
  done
done
cat gpurun_out/pmc/summary_fp8.txt
