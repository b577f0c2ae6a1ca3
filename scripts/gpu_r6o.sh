#!/bin/bash
# round 6 final-tree profiles: headline (bench.py --steps 2), serving load test, config 2 encoder
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_profile.sh || exit $?
grep -o '"value": [0-9.]*\|"decode_plan": {[^}]*}' gpurun_out/prof_bench.log
bash scripts/gpu_profile_serve.sh || exit $?
bash scripts/gpu_prof_encoder.sh || exit $?
