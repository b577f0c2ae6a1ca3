#!/bin/bash
# Round 4: EP-vs-TP MoE layer probe (config-5 shapes, one rank each, rocprofv3 kernel stats), then the
# headline bench profile (rocprofv3 --kernel-trace --stats of bench.py --steps 2 --warmup 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p gpurun_out/prof_ep
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python3 -u scripts/ep_probe.py 2048 20 > gpurun_out/ep_probe.log 2>&1
rc=$?; echo "ep_probe rc=$rc"; grep -v amdgpu.ids gpurun_out/ep_probe.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ep -o run -- \
    python3 scripts/ep_probe.py 2048 20 > gpurun_out/ep_probe_prof.log 2>&1
rc=$?; echo "ep rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
STATS=$(find gpurun_out/prof_ep -name "*kernel_stats.csv" | head -1)
[ -n "$STATS" ] && python3 scripts/summarize_profile.py "$STATS" "scripts/ep_probe.py 2048 20 (rocprofv3)" \
    gpurun_out/prof_ep_summary.md > /dev/null
find gpurun_out/prof_ep -name "*kernel_trace.csv" -delete
bash scripts/gpu_profile.sh
