#!/bin/bash
# rocprofv3 kernel-trace + stats of the serving load test (scripts/serve_load.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_serve
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serve -o run -- \
    python3 scripts/serve_load.py --requests ${SERVE_N:-192} --concurrency 64 > gpurun_out/prof_serve.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep "score requests" gpurun_out/prof_serve.log | cut -c1-300
STATS=$(find gpurun_out/prof_serve -name "*kernel_stats.csv" | head -1)
[ -n "$STATS" ] && python3 scripts/summarize_profile.py "$STATS" "serve_load.py (rocprofv3 --kernel-trace --stats)" \
    gpurun_out/prof_serve_summary.md > /dev/null
TRACE=$(find gpurun_out/prof_serve -name "*kernel_trace.csv" | head -1)
[ -n "$TRACE" ] && python3 scripts/trace_shapes.py "$TRACE" 40 > gpurun_out/prof_serve_shapes.md
find gpurun_out/prof_serve -name "*kernel_trace.csv" -delete
exit $rc
