#!/bin/bash
# PMC counters of gemm4w (both DMA splits) vs hipBLASLt on one shape (run via gpurun).  Each rocprofv3 run
# is its own process with its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$R"
SHAPE=${SHAPE:-"4096 4096 4096"}
for kind in ${KINDS:-g4s0 g4s1 blas}; do
  case $kind in g4s0) export LWC_G4_SPLIT=0; k=g4;; g4s1) export LWC_G4_SPLIT=1; k=g4;; *) k=$kind;; esac
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" ; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc/${kind}_${tag} -o run -- \
      python3 scripts/gemm_probe.py $k $SHAPE 10 > gpurun_out/pmc/${kind}_${tag}.log 2>&1 || exit 1
    echo "## $kind" >> gpurun_out/pmc/summary_g4.txt
    python3 scripts/pmc_summary.py /tmp/pmc/${kind}_${tag} >> gpurun_out/pmc/summary_g4.txt 2>&1
  done
done
cat gpurun_out/pmc/summary_g4.txt
