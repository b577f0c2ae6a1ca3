#!/bin/bash
# rocprofv3 kernel-trace + stats of the config-5 bench (Mixtral fp8 sampler + e5-mistral embedder).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_moe
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_moe -o run -- \
    python3 bench_configs.py moe --requests ${MOE_R:-8} --steps 1 --warmup 1 > gpurun_out/prof_moe.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -v "rocprofv3\|output_stream\|simple_timer" gpurun_out/prof_moe.log | tail -3 | cut -c1-300
STATS=$(find gpurun_out/prof_moe -name "*kernel_stats.csv" | head -1)
[ -n "$STATS" ] && python3 scripts/summarize_profile.py "$STATS" "bench_configs.py moe (rocprofv3 --kernel-trace --stats)" \
    gpurun_out/prof_moe_summary.md > /dev/null
find gpurun_out/prof_moe -name "*kernel_trace.csv" -delete
exit $rc
