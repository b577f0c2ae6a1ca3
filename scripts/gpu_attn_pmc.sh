#!/bin/bash
# PMC counters of the cascade decode attention (scripts/attn_probe.py), one rocprofv3 pass per counter set.
# ATTN_SETS overrides the sets ("|"-separated); ATTN_MODE = full | suffix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MODE=${ATTN_MODE:-suffix}
SUM=gpurun_out/pmc/attn_summary_${MODE}.txt
: > $SUM
SETS=${ATTN_SETS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAVES|GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum|TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"}
IFS='|' read -ra ARR <<< "$SETS"
for set in "${ARR[@]}"; do
  tag=$(echo $set | cut -d' ' -f1)
  rm -rf /tmp/pmc/attn_${tag}
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc/attn_${tag} -o run -- \
    python3 scripts/attn_probe.py 64 10 $MODE > gpurun_out/pmc/attn_${tag}.log 2>&1 || exit 1
  python3 - /tmp/pmc/attn_${tag} >> $SUM <<'PY'
import csv, glob, sys
from collections import defaultdict
per, disp = defaultdict(float), set()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "cascade" in r.get("Kernel_Name", ""):
            per[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r.get("Dispatch_Id", ""))
n = max(1, len(disp))
for c, v in sorted(per.items()):
    print(f"{c:28s} {v / n:16.0f}")
PY
done
cat $SUM
