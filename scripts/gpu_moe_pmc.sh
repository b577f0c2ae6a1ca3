#!/bin/bash
# PMC counters of the fp8 MoE grouped GEMM (scripts/moe_probe.py), one rocprofv3 pass per counter set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SUM=gpurun_out/pmc/moe_summary_${LWC_MOE_GEMM:-auto}_T${MOE_T:-512}.txt
: > $SUM
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVES" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  tag=$(echo $set | cut -d' ' -f1)
  rm -rf /tmp/pmc/moe_${tag}
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc/moe_${tag} -o run -- \
    python3 scripts/moe_probe.py ${MOE_T:-512} 10 > gpurun_out/pmc/moe_${tag}.log 2>&1 || exit 1
  python3 - /tmp/pmc/moe_${tag} >> $SUM <<'PY'
import csv, glob, sys
from collections import defaultdict
per, disp = defaultdict(float), set()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "grouped_gemm" in r.get("Kernel_Name", "") or "gemm8g" in r.get("Kernel_Name", ""):
            per[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r.get("Dispatch_Id", ""))
n = max(1, len(disp))
for c, v in sorted(per.items()):
    print(f"{c:28s} {v / n:16.0f}")
PY
done
cat $SUM
