#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here; those go in their own run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1"}
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py $ARGS > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -5 gpurun_out/prof_bench.log
STATS=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
[ -n "$STATS" ] && python3 scripts/summarize_profile.py "$STATS" "bench.py $ARGS (rocprofv3 --kernel-trace --stats)" \
    gpurun_out/prof_summary.md > /dev/null
# GPU idle gaps (host stalls) over the whole run, before the trace is dropped
TRACE=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
[ -n "$TRACE" ] && python3 scripts/trace_gaps.py "$TRACE" ${GAP_MS:-0.2} > gpurun_out/prof_gaps.txt
# per call site (kernel, predecessor): separates the library's o / down / lm_head calls
[ -n "$TRACE" ] && python3 scripts/trace_shapes.py "$TRACE" 40 > gpurun_out/prof_shapes.md
# keep the stats, drop the multi-MB per-dispatch trace (gpurun copies back <= 64 MiB)
find gpurun_out/prof -name "*kernel_trace.csv" -delete
exit $rc
