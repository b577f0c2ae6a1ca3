#!/bin/bash
# Multi-rank rehearsal on a ONE-GPU box: 2 ranks share GPU 0, collectives over gloo (LWC_SHARE_ONE_GPU=1).
# Exercises the candidate-parallel bench path (export_prefill -> all-gather prompt KV -> import ->
# decode -> all-gather embeddings -> consensus) end to end.  Real RCCL runs happen on 8-GPU nodes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
NP=${REH_W:-2}
LWC_SHARE_ONE_GPU=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $NP --steps 1 --warmup 1 \
  --requests ${REH_R:-4} --profile-steps ${REH_ARGS:-} > gpurun_out/rehearsal.log 2>&1
rc=$?; echo "rehearsal rc=$rc"; grep -v amdgpu.ids gpurun_out/rehearsal.log | tail -8
[ $rc -eq 0 ] || exit $rc
# the same through bench.py's own launcher (no torchrun): `python bench.py --gpus N`
LWC_SHARE_ONE_GPU=1 timeout -k 10 900 python bench.py --gpus $NP --steps 1 --warmup 1 --requests ${REH_R:-4} \
  > gpurun_out/rehearsal_selflaunch.log 2>&1
rc=$?; echo "self-launch rehearsal rc=$rc"; grep -v amdgpu.ids gpurun_out/rehearsal_selflaunch.log | tail -4
exit $rc
