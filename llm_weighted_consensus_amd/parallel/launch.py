"""Self-launch of one process per GPU for the bench entry points (``bench.py --gpus N``,
``bench_configs.py moe --tp 2``).

When a script is started directly with ``--gpus N > 1`` and no torchrun env (``WORLD_SIZE`` unset), the
parent process becomes a pure launcher: it NEVER touches the GPU (no HIP call, no
``torch.cuda.is_available()``), picks a free rendezvous port on 127.0.0.1, starts N children of the same
script with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, and exits
with the worst child status.  Children are separate processes (never ``exec``: a GPU-initialised
process must not be replaced).  If any rank fails, the others are terminated so a rank stuck in a
collective does not hold the node.  Under torchrun (``WORLD_SIZE`` set) this is a no-op.

The reference fans one request out to many upstream voters concurrently
(/root/reference/src/score/completions/client.rs:343-356); on MI355X the fan-out is a candidate-parallel
process group over RCCL, one process per GPU.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def child_env(rank: int, world: int, port: int, base: Optional[dict] = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # dmabuf IPC is the only mode the host driver supports (RCCL peer buffers, CUDA-tensor sharing)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def launch(world: int, argv: Sequence[str], poll_s: float = 0.2) -> int:
    """Run ``argv`` as ``world`` ranks; return 0 when every rank exits 0, else the first non-zero status
    (a rank killed by a signal reports 128 + signal)."""
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(world):
        procs.append(subprocess.Popen(list(argv), env=child_env(r, world, port)))
    # one waiter thread per rank records exits in the order they happen: the first failure is the
    # cause, the ranks that then lose their peers (and fail too) are not
    exits: List[tuple] = []
    lock = threading.Lock()

    def waiter(r: int) -> None:
        rc = procs[r].wait()
        with lock:
            exits.append((time.monotonic(), r, rc))

    for r in range(world):
        threading.Thread(target=waiter, args=(r,), daemon=True).start()
    status = 0
    try:
        seen = 0
        while seen < world:
            with lock:
                new = sorted(exits)[seen:] if len(exits) > seen else []
            for _, r, rc in new:
                seen += 1
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"launch: rank {r} exited with {rc}; stopping the other ranks", file=sys.stderr)
                    for q in range(world):
                        if procs[q].poll() is None:
                            procs[q].send_signal(signal.SIGTERM)
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return status


def maybe_self_launch(gpus: int, script: str) -> Optional[int]:
    """Called FIRST in a bench entry point.  Returns None when this process is a rank (run the bench),
    or the launcher's exit status when it started ``gpus`` ranks itself (the caller exits with it)."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    return launch(gpus, [sys.executable, "-u", os.path.abspath(script)] + sys.argv[1:])


def check_world(expected: int, got: int) -> None:
    """The whole-node metric must never be reported from a silently smaller world."""
    if expected != got:
        raise SystemExit(f"--gpus {expected} but the process group has world size {got}: refusing to report "
                         f"a {got}-rank number as an {expected}-GPU one")
