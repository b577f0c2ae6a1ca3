"""Process-group bring-up and the collectives the framework uses (RCCL over xGMI on MI355X).

One process per GPU; `torch.distributed` backend "nccl" IS RCCL on ROCm.  On CPU (tests) the same
code runs over gloo.  Collectives used by the serving/bench paths:

  C1 all_gather of candidate embeddings  [n_local, d] -> [world, n_local, d]
  C2 voter shares / votes                leader <-> follower TCP links, not collectives: a dead peer must
                                         cost its voters, not the request (parallel/shard_link.py,
                                         score/sharded.py)
  C3 TP all-reduce                       (tensor-parallel decoders; IPC one-shot kernel, parallel/allreduce.py)
  C4 all_to_all_single                   (expert-parallel MoE dispatch / combine, parallel/expert.py)
  C5 broadcast / barrier                 (control)

xGMI on MI355X is point-to-point (7 links per GPU): the payloads here are small (an all-gather of
64 x 1024 bf16 = 128 KiB per rank), i.e. latency-bound, so we issue ONE collective per phase on a
flat buffer instead of many small ones.
"""
from __future__ import annotations

import datetime
import os
import time
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: Optional[str] = None

    @property
    def enabled(self) -> bool:
        return self.world > 1


_INFO = DistInfo()


def init_from_env(device_type: Optional[str] = None, timeout_s: Optional[float] = None) -> DistInfo:
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/
    MASTER_ADDR/MASTER_PORT).  Single-process when WORLD_SIZE is unset or 1.

    ``LWC_SHARE_ONE_GPU=1`` is a rehearsal mode for one-GPU boxes: every rank uses GPU 0 and the
    collectives run over gloo (staged through host memory), so the multi-rank code paths can be
    exercised end to end where RCCL cannot put two ranks on one device."""
    global _INFO
    if timeout_s is None:
        timeout_s = float(os.environ.get("LWC_COLLECTIVE_TIMEOUT_S", "600"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    share = os.environ.get("LWC_SHARE_ONE_GPU") == "1"
    if share:
        local = 0
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if device_type == "cuda" and not share else "gloo"
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(**kw)
        _INFO = DistInfo(rank, world, local, backend)
    else:
        _INFO = DistInfo(rank, world, local, dist.get_backend() if dist.is_initialized() else None)
    return _INFO


def info() -> DistInfo:
    return _INFO


def barrier() -> None:
    if _INFO.enabled:
        if _INFO.backend == "nccl":
            dist.barrier(device_ids=[_INFO.local_rank])
        else:
            dist.barrier()


def group_size(group=None) -> int:
    return dist.get_world_size(group) if _INFO.enabled else 1


# Per-collective accounting (bench JSON at W > 1): tag -> calls, bytes this rank receives, and the
# (start, end) events bracketing each call on the issuing stream; ms are read once, after a synchronize
_COMM: dict = {}
_TAG: list = [None]


class comm_tag:
    """``with comm_tag("C1"):`` — the collectives issued inside count under that tag (:func:`comm_report`)."""

    def __init__(self, tag: str):
        self.tag = tag

    def __enter__(self):
        self.prev, _TAG[0] = _TAG[0], self.tag
        return self

    def __exit__(self, *exc):
        _TAG[0] = self.prev
        return False


def _comm_begin(nbytes: int, device):
    tag = _TAG[0]
    if tag is None:
        return None
    rec = _COMM.setdefault(tag, {"calls": 0, "bytes": 0, "events": []})
    rec["calls"] += 1
    rec["bytes"] += int(nbytes)
    if device is not None and device.type == "cuda":
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        return rec, e0
    return rec, time.perf_counter()


def _comm_end(tok) -> None:
    if tok is None:
        return
    rec, start = tok
    if isinstance(start, float):
        rec["events"].append((start, time.perf_counter()))
    else:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        rec["events"].append((start, e1))


def comm_report(steps: int = 1, reset: bool = True) -> dict:
    """{tag: {"calls", "bytes", "ms"}} per step (divided by ``steps``) of the tagged collectives since the last
    reset; synchronizes the device first (call outside timed regions or at their end)."""
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    out = {}
    for tag, rec in _COMM.items():
        ms = 0.0
        for a, b in rec["events"]:
            ms += (b - a) * 1e3 if isinstance(a, float) else a.elapsed_time(b)
        n = max(1, steps)
        out[tag] = {"calls": rec["calls"] / n, "bytes": rec["bytes"] // n, "ms": round(ms / n, 3)}
    if reset:
        _COMM.clear()
    return out


def all_gather_flat(t: torch.Tensor, group=None) -> torch.Tensor:
    """[*] per rank -> [group size, *]: one all_gather_into_tensor on the flattened buffer (the 1-D form
    works for RCCL and gloo alike; GPU tensors under gloo are staged through host memory)."""
    W = group_size(group)
    tok = _comm_begin(W * t.numel() * t.element_size(), t.device)
    try:
        return _all_gather_flat(t, W, group)
    finally:
        _comm_end(tok)


def _all_gather_flat(t: torch.Tensor, W: int, group=None) -> torch.Tensor:
    flat = t.contiguous().view(-1)
    if _INFO.backend == "gloo" and flat.is_cuda:
        host = flat.cpu()
        out = torch.empty(W * host.numel(), dtype=host.dtype)
        dist.all_gather_into_tensor(out, host, group=group)
        return out.to(t.device).view(W, *t.shape)
    out = torch.empty(W * flat.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, flat, group=group)
    return out.view(W, *t.shape)


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None,
                      group=None) -> torch.Tensor:
    """All-to-all along dim 0 (C4, expert-parallel dispatch/combine): equal splits when the split lists
    are None.  GPU tensors under gloo are staged through host memory (one-GPU rehearsal mode)."""
    if not _INFO.enabled:
        out.copy_(inp)
        return out
    if _INFO.backend == "gloo":
        # host staging; dtypes gloo does not reduce over (bf16, fp8) travel as raw bytes per row
        h_in = inp.detach().cpu().contiguous()
        h = torch.empty(out.shape, dtype=out.dtype)
        if h_in.dtype not in (torch.float32, torch.float64, torch.int32, torch.int64, torch.uint8):
            row = 1
            for n in h_in.shape[1:]:
                row *= n
            bi = h_in.reshape(h_in.shape[0], row).view(torch.uint8)
            bo = h.view(h.shape[0], row).view(torch.uint8)
            dist.all_to_all_single(bo, bi, out_splits, in_splits, group=group)
        else:
            dist.all_to_all_single(h, h_in, out_splits, in_splits, group=group)
        out.copy_(h)
        return out
    if inp.dtype == torch.float8_e4m3fn:  # e4m3 rows travel as bytes
        dist.all_to_all_single(out.view(torch.uint8), inp.contiguous().view(torch.uint8), out_splits, in_splits,
                               group=group)
        return out
    dist.all_to_all_single(out, inp.contiguous(), out_splits, in_splits, group=group)
    return out


def all_gather(t: torch.Tensor, group=None) -> torch.Tensor:
    """[*] per rank -> [group size, *] (C1).  One collective on a contiguous buffer."""
    if not _INFO.enabled:
        return t.unsqueeze(0)
    return all_gather_flat(t, group)


def candidate_groups(cp: int):
    """Split the world into world/cp consecutive groups of cp ranks (candidate-parallel inside a group,
    request-parallel across groups).  Every rank creates every group (collective), returns
    (this rank's group handle or None when cp == 1 / single process, group index, rank in group)."""
    if not _INFO.enabled:
        return None, 0, 0
    W, r = _INFO.world, _INFO.rank
    if cp < 1 or W % cp:
        raise ValueError(f"candidate-parallel degree {cp} must divide the world size {W}")
    mine = None
    for d in range(W // cp):
        g = dist.new_group(ranks=list(range(d * cp, (d + 1) * cp)))
        if d == r // cp:
            mine = g
    return (mine if cp > 1 else None), r // cp, r % cp


def all_reduce_(t: torch.Tensor, op: str = "sum", group=None) -> torch.Tensor:
    """In-place all-reduce (C3 for tensor parallelism, or control reductions)."""
    if _INFO.enabled:
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        if _INFO.backend == "gloo" and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, op=rop, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=rop, group=group)
    return t


def max_over_ranks(x: float, device=None) -> float:
    if not _INFO.enabled:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    all_reduce_(t, "max")
    return float(t.item())


def world_size_seen() -> int:
    """Number of ranks that take part in one all-reduce of ones on the default group (collective; on
    RCCL the tensor lives on this rank's GPU).  Reported in the bench line so a whole-node number can be
    checked against the world the backend actually formed."""
    if not _INFO.enabled:
        return 1
    dev = torch.device("cuda", _INFO.local_rank) if _INFO.backend == "nccl" else torch.device("cpu")
    t = torch.ones(1, dtype=torch.int32, device=dev)
    dist.all_reduce(t)
    return int(t.item())


def broadcast_object(obj, src: int = 0, group=None):
    """``obj`` of group rank ``src`` on every rank of ``group`` (default: the world)."""
    if group is None and not _INFO.enabled:
        return obj
    lst = [obj]
    gsrc = dist.get_global_rank(group, src) if group is not None else src
    dist.broadcast_object_list(lst, src=gsrc, group=group)
    return lst[0]


class CollectiveFailure(RuntimeError):
    """A collective failed (peer died, timeout, transport error); the process group has been aborted and
    this process continues single-rank (``info().enabled`` is now False)."""


def abort() -> None:
    """Tear the process group down after a failed collective WITHOUT waiting on peers (a dead peer would
    hang a graceful destroy), and continue as a single rank.  RCCL communicators are aborted by the
    backend's own abort; gloo just drops its sockets."""
    global _INFO
    if dist.is_initialized():
        try:
            pg = dist.distributed_c10d._get_default_group()
            if hasattr(pg, "abort"):
                pg.abort()
        except Exception:  # noqa: BLE001 - best effort: the group is being discarded
            pass
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass
    _INFO = DistInfo(_INFO.rank, 1, _INFO.local_rank, None)


_TRANSPORT_MARKERS = ("gloo", "transport", "nccl", "rccl", "timed out", "timeout", "connection", "closed by peer", "socket",
                      "abort", "broken pipe", "reset by peer", "watchdog")


def is_transport_error(e: BaseException) -> bool:
    """True for failures of the collective transport itself (dead or hung peer, socket / RCCL error,
    process-group timeout).  Local bugs — OOM, shape / dtype mismatches, bad arguments — are NOT: they
    propagate unchanged and the process group stays up."""
    if isinstance(e, torch.OutOfMemoryError):
        return False
    if isinstance(e, (dist.DistError, TimeoutError, ConnectionError)):
        return True
    if type(e) is RuntimeError:
        msg = str(e).lower()
        return any(m in msg for m in _TRANSPORT_MARKERS)
    return False


def guarded(fn, *args, fallback=None, **kw):
    """Run a collective; on a TRANSPORT failure (:func:`is_transport_error`) abort the group (see
    :func:`abort`) and return ``fallback()`` (or raise :class:`CollectiveFailure` when no fallback is
    given).  Any other exception is re-raised untouched.  Failure detection is the process group's own
    timeout (``init_from_env(timeout_s=...)``, ``LWC_COLLECTIVE_TIMEOUT_S``) plus the transport noticing a
    dead peer — whichever comes first."""
    try:
        return fn(*args, **kw)
    except Exception as e:  # noqa: BLE001 - classified below
        if not is_transport_error(e):
            raise
        abort()
        if fallback is None:
            raise CollectiveFailure(f"collective {getattr(fn, '__name__', fn)} failed: {e}") from e
        return fallback()


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
