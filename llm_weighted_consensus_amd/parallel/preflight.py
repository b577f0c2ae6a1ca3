"""Start-up pre-flight of a multi-GPU run (world > 1): make the first 8-GPU measurement explain itself.

Before the benches' first step every rank checks, collectively:

* **peer access** — ``hipDeviceCanAccessPeer`` from this rank's device to every other visible device
  (``torch.cuda.can_device_access_peer``), gathered into the whole matrix on every rank;
* **RCCL all-gather** — one all-gather of a known tensor (rank r contributes r + 1 in every element) through
  the process group, every chunk checked, timed;
* **IPC collectives** (only when the run asked for them, ``want_ipc``) — the one-shot IPC all-reduce's own
  start-up self-test against the process group (``CustomAllReduce``).  If any peer pair lacks access, or the
  self-test fails, the IPC path is not used and the reason is returned (``ipc_fallback``): the caller runs its
  collectives on RCCL instead.

The result goes into the bench JSON (``preflight``) together with per-step bytes / milliseconds of the tagged
collectives (C1 embeddings, C4 prompt KV: ``dist.comm_report``), so a bad scaling number can be traced to a
missing peer path, a slow collective or the compute.  The reference runs no collectives (its fan-out is HTTP,
``/root/reference/src/score/completions/client.rs:343-356``); this serves the candidate-parallel layout.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch
import torch.distributed as dist

from . import dist as pdist


def peer_matrix(device: torch.device) -> list:
    """This rank's row: can ``device`` access every visible device (True on the diagonal)?"""
    if device.type != "cuda":
        return []
    n = torch.cuda.device_count()
    me = device.index if device.index is not None else torch.cuda.current_device()
    return [True if j == me else bool(torch.cuda.can_device_access_peer(me, j)) for j in range(n)]


def run(device: torch.device, group=None, want_ipc: bool = False, force_peer_fail: Optional[bool] = None) -> dict:
    """Collective over ``group`` (default: the world).  Returns {"world_size_rccl", "backend", "devices",
    "peer_access" ("all" or the list of missing pairs), "rccl_allgather" ({ok, ms, bytes}), "ipc"
    ("not requested" / "ok" / "fallback: <reason>"), "ipc_fallback" (bool)}.  ``force_peer_fail``
    (or ``LWC_PREFLIGHT_FORCE_PEER_FAIL=1``) pretends a pair lacks peer access: the fallback path, tested."""
    W = dist.get_world_size(group)
    rank = dist.get_rank(group)
    backend = dist.get_backend(group)
    if force_peer_fail is None:
        force_peer_fail = os.environ.get("LWC_PREFLIGHT_FORCE_PEER_FAIL") == "1"
    # peer matrix: one object all-gather of (rank, device index, row)
    row = peer_matrix(device)
    rows = [None] * W
    dist.all_gather_object(rows, (rank, device.index if device.type == "cuda" else -1, row), group=group)
    devs = [r[1] for r in rows]
    missing = []
    for r, d, rw in rows:
        for r2, d2, _ in rows:
            if d >= 0 and d2 >= 0 and d != d2 and (d2 >= len(rw) or not rw[d2]):
                missing.append(f"{d}->{d2}")
    if force_peer_fail:
        missing.append("forced (LWC_PREFLIGHT_FORCE_PEER_FAIL)")
    # RCCL (or gloo) all-gather of a known tensor, checked and timed
    on_dev = backend == "nccl"
    x = torch.full((1 << 16,), float(rank + 1), dtype=torch.float32, device=device if on_dev else "cpu")
    out = torch.empty(W * x.numel(), dtype=x.dtype, device=x.device)
    if on_dev:
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    dist.all_gather_into_tensor(out, x, group=group)
    if on_dev:
        torch.cuda.synchronize(device)
    ms = (time.perf_counter() - t0) * 1e3
    want = torch.arange(1, W + 1, dtype=torch.float32, device=out.device).repeat_interleave(x.numel())
    ok = bool(torch.equal(out, want))
    flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=x.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    ag_ok = int(flag.item()) == 0
    res = {"world_size_rccl": W, "backend": backend, "devices": devs,
           "peer_access": "all" if not missing else missing,
           "rccl_allgather": {"ok": ag_ok, "ms": round(ms, 3), "bytes": int(out.numel() * 4)},
           "ipc": "not requested", "ipc_fallback": False}
    if not ag_ok:
        raise RuntimeError(f"pre-flight: the process group's all-gather returned wrong data on some rank: {res}")
    if want_ipc:
        if missing:
            res["ipc"], res["ipc_fallback"] = f"fallback: no peer access on {', '.join(missing[:8])}", True
        elif not on_dev or device.type != "cuda":
            res["ipc"], res["ipc_fallback"] = "fallback: the IPC collectives need an RCCL group on GPUs", True
        else:
            from .allreduce import CommFailure, CustomAllReduce

            try:
                ar = CustomAllReduce(group, device, max_bytes=1 << 20, self_test=True)
                ar.close()
                res["ipc"] = "ok"
            except (CommFailure, RuntimeError) as e:
                res["ipc"], res["ipc_fallback"] = f"fallback: IPC self-test failed ({e})", True
        # every rank must take the same path
        f = torch.tensor([1 if res["ipc_fallback"] else 0], dtype=torch.int32, device=x.device)
        dist.all_reduce(f, op=dist.ReduceOp.MAX, group=group)
        if int(f.item()) and not res["ipc_fallback"]:
            res["ipc"], res["ipc_fallback"] = "fallback: another rank's IPC check failed", True
    return res


def maybe_run(device: torch.device, want_ipc: bool = False) -> Optional[dict]:
    """:func:`run` over the world when this is a multi-rank run, else None."""
    info = pdist.info()
    if not info.enabled or info.world < 2:
        return None
    return run(device, None, want_ipc=want_ipc)
