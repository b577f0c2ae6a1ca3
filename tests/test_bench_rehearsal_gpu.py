"""The multi-rank headline bench path end to end on ONE GPU: ``bench.py --gpus 2`` self-launches two
ranks that share the card (LWC_SHARE_ONE_GPU=1: gloo collectives), with a tiny decoder / encoder.  It runs
what the driver's N = 2..8 scaling runs run — the launcher, candidate-parallel groups (cp = 2), the prompt
KV + last-logit all-gather (C4), the embedding all-gather (C1), the consensus, max-over-ranks timing — and
prints the one JSON line.  RCCL over xGMI itself is covered by tests/test_rccl_gpu.py on a multi-GPU box."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_share_one_gpu(gpu):
    env = dict(os.environ, LWC_SHARE_ONE_GPU="1", MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--decoder", "llama-tiny",
           "--encoder", "bert-tiny", "--steps", "1", "--warmup", "1", "--requests", "2", "--candidates", "64",
           "--prompt-len", "32", "--gen-len", "8"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["value"] > 0 and out["steps"] == 1 and out["world_size"] == 2
    assert out["n_gpus"] == 1  # shared card: never reported as a 2-GPU number
    assert out["config"]["global_batch"] == 4 and "cp2" in out["config"]["parallelism"]
