#!/bin/bash
# A/B of environment settings on ONE box: bench.py --steps 2 --warmup 1 per setting, interleaved twice.
# Usage: bash scripts/gpu_ab.sh "LWC_X=0" "LWC_X=1" ...   (each argument: space-separated VAR=value list; "" = default)
# AB_CMD replaces the bench command (e.g. AB_CMD="python3 -u scripts/serve_load.py --requests 256"; its JSON
# line's "value" is reported the same way)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROUNDS=${AB_ROUNDS:-2}
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    log=gpurun_out/ab_${i}_r${r}.log
    timeout -k 10 600 env $setting ${AB_CMD:-python3 bench.py --steps ${AB_STEPS:-2} --warmup 1 ${AB_ARGS}} > "$log" 2>&1
    rc=$?
    v=$(grep -o '"value": [0-9.]*\|"p99": [0-9.]*' "$log" | head -2 | tr '\n' ' ')
    echo "round $r [$setting] rc=$rc $v"
    [ $rc -eq 0 ] || exit $rc
  done
done
