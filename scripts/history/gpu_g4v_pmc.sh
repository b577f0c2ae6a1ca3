#!/bin/bash
# PMC counters of the gemm4w main loops (LWC_G4_VAR 1: BK 64 two buffers; 16: BK 32 five-slot ring) vs
# hipBLASLt on one shape.  One rocprofv3 run per counter set, each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$R"
SHAPE=${SHAPE:-"4096 4096 14336"}
rm -f gpurun_out/pmc/summary_g4v.txt
for kind in ${KINDS:-v1 v16 blas}; do
  case $kind in v1) export LWC_G4_VAR=1; k=g4;; v16) export LWC_G4_VAR=16; k=g4;; *) k=$kind;; esac
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU" \
             ; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc/${kind}_${tag} -o run -- \
      python3 scripts/gemm_probe.py $k $SHAPE 10 > gpurun_out/pmc/${kind}_${tag}.log 2>&1 || { echo "pmc $kind $tag failed"; tail -5 gpurun_out/pmc/${kind}_${tag}.log; continue; }
    echo "## $kind" >> gpurun_out/pmc/summary_g4v.txt
    python3 scripts/pmc_summary.py /tmp/pmc/${kind}_${tag} >> gpurun_out/pmc/summary_g4v.txt 2>&1
  done
done
cat gpurun_out/pmc/summary_g4v.txt
