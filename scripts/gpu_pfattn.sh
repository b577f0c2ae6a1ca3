set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 python -u scripts/microbench.py pfattn > gpurun_out/pfattn.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/pfattn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pfattn -o run -- python -u scripts/microbench.py pfattn > gpurun_out/pfattn_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; f=$(find gpurun_out/prof_pfattn -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
exit $rc
