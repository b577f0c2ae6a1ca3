set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for bk in 0 1 0 1; do
  LWC_GEMM_BUCKETS=$bk timeout -k 10 300 python3 -u scripts/serve_load.py --requests 256 --concurrency 64 > gpurun_out/serve_bk$bk.log 2>&1
  rc=$?; echo "buckets=$bk rc=$rc"; grep '"metric"' gpurun_out/serve_bk$bk.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
