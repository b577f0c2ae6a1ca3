#!/bin/bash
# rocprofv3 kernel-trace + stats of one scripts/microbench.py section: bash scripts/gpu_prof_micro.sh <what>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
W=${1:-route}
mkdir -p gpurun_out/prof_micro_$W
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_micro_$W -o run -- \
    python3 scripts/microbench.py $W > gpurun_out/prof_micro_$W.log 2>&1
rc=$?; echo "rocprof rc=$rc"
STATS=$(find gpurun_out/prof_micro_$W -name "*kernel_stats.csv" | head -1)
[ -n "$STATS" ] && python3 scripts/summarize_profile.py "$STATS" "microbench.py $W (rocprofv3 --kernel-trace --stats)" \
    gpurun_out/prof_micro_${W}_summary.md > /dev/null
find gpurun_out/prof_micro_$W -name "*kernel_trace.csv" -delete
exit $rc
