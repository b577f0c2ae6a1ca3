#!/bin/bash
# One GPU call = one or more named tasks, each under its own time limit, chained so the first failure ends
# the call.  Usage (through gpurun):  bash scripts/gpu_task.sh <task> [<task> ...]
#   suite         the whole GPU test suite
#   smoke         __graft_entry__.smoke()
#   bench         the driver's bench command (BENCH_ARGS overrides: default --steps 20 --warmup 5)
#   quick         bench.py --steps 2 --warmup 1 --profile-steps ($QUICK_ARGS appended)
#   prof          rocprofv3 kernel-trace + stats of bench.py (scripts/gpu_profile.sh; BENCH_ARGS)
#   g4ab          scripts/microbench.py g4ab (G4_SHAPES / G4_VARS select)
#   kernels       tests/test_kernels_gpu.py (-k $KSEL)
#   pytest:<path> one test file / node id
#   micro:<what>  scripts/microbench.py <what>
#   configs       bench_configs.py encoder + moe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python3 -u -m pytest -x -q -p no:cacheprovider --timeout-method thread"
step() {  # step <name> <seconds> <cmd...>: output to gpurun_out/<name>.log, tail on stdout
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
for t in "$@"; do
  case "$t" in
    suite) step suite 1000 $PYT --timeout 300 -m gpu tests || exit $? ;;
    smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) step bench 900 python3 bench.py --gpus 1 ${BENCH_ARGS:---steps 20 --warmup 5} || exit $? ;;
    quick) step quick 900 python3 bench.py --steps 2 --warmup 1 --profile-steps $QUICK_ARGS || exit $? ;;
    prof) bash scripts/gpu_profile.sh || exit $? ;;
    g4ab) step g4ab 900 python3 scripts/microbench.py g4ab || exit $? ;;
    kernels) step kernels 900 $PYT --timeout 120 -m gpu tests/test_kernels_gpu.py -k "${KSEL:-.}" || exit $? ;;
    pytest:*) step "pytest_$(basename "${t#pytest:}" | tr ':[]/' '____')" 900 $PYT --timeout 200 -m gpu "${t#pytest:}" || exit $? ;;
    micro:*) step "micro_${t#micro:}" 900 python3 scripts/microbench.py ${t#micro:} || exit $? ;;
    configs) step cfg_encoder 900 python3 bench_configs.py encoder --steps 2 || exit $?
             step cfg_moe 900 python3 bench_configs.py moe --steps 2 || exit $? ;;
    *) echo "unknown task $t"; exit 2 ;;
  esac
done
