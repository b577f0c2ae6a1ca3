#!/bin/bash
# rocprofv3 kernel-trace + stats of config 2 (bench_configs.py encoder --steps 2): where the encoder step goes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_enc
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_enc -o run -- \
    python3 bench_configs.py encoder --steps 2 > gpurun_out/prof_enc.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/prof_enc.log
STATS=$(find gpurun_out/prof_enc -name "*kernel_stats.csv" | head -1)
[ -n "$STATS" ] && python3 scripts/summarize_profile.py "$STATS" "bench_configs.py encoder --steps 2 (rocprofv3 --kernel-trace --stats)" \
    gpurun_out/prof_enc_summary.md > /dev/null
find gpurun_out/prof_enc -name "*kernel_trace.csv" -delete
exit $rc
