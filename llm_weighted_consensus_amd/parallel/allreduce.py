"""C3: one-shot tensor-parallel all-reduce over IPC-mapped peer buffers (csrc/kernels/allreduce.hip).

Each rank allocates one uncached device REGION, exports its IPC handle, and the handles are exchanged
once over the process group (a host-side all_gather_object — gloo or RCCL alike); every rank then maps
every peer's region.  ``all_reduce_(x)`` is a single kernel launch on the current stream (no host
synchronisation, no RCCL call), so a tensor-parallel decode step captures into one hipGraph with its
all-reduces inside.  Ranks sum in rank order, so every rank holds bitwise-identical results.

xGMI is point-to-point: at TP=2 a one-shot push moves each activation over the one link between the
pair exactly once per direction, the minimum for any all-reduce algorithm; the win over RCCL is launch
latency and graph capture (RCCL's eager call is ~20-40 us host-side per call, 64 calls per step).

The reference has no tensor parallelism (it runs no model); this serves BASELINE config 5 (Mixtral
TP=2) in place of the round-1 eager ``dist.all_reduce``.

Start-up self-test: the constructor (a collective) runs one call on a random tensor and compares it with
the same reduction through the process group (an all-gather of every rank's input, summed in fp32 on the
host); a mismatch or a raised error word raises :class:`CommFailure` before the first request, so a broken
peer mapping (cross-device ``hipIpcOpenMemHandle``, xGMI coherence of the uncached region) fails loudly at
bring-up instead of decoding garbage.  ``LWC_AR_SELFTEST=0`` skips it.

Failure: a peer that does not arrive within the spin bound (``spin_ms``, env ``LWC_AR_SPIN_MS``; the
kernel's default is ~4 s) makes the waiting rank poison its output with NaN and set a sticky device
error word — never sum a stale slot.  The engine reads that word without a host sync: :meth:`arm` queues
a copy of it into pinned memory behind each decode step, and :meth:`poll` (called once the step's
outputs are on the host, i.e. one step later) raises :class:`CommFailure`, which fails the in-flight
requests (``EngineService`` -> ``EngineFailure``) instead of letting NaN logits decode on.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import ops


class CommFailure(RuntimeError):
    """A tensor-parallel peer never arrived at an all-reduce (spin bound exceeded)."""


# one poll iteration of the kernel's wait loop is an s_sleep(2) plus a system-scope load: ~60 ns
_NS_PER_SPIN = 60


class CustomAllReduce:
    def __init__(self, group=None, device=None, max_bytes: int = 64 << 20, blocks: int = 128,
                 spin_ms: Optional[float] = None, self_test: Optional[bool] = None):
        """Collective: every rank of ``group`` (default: the world) must construct it together.
        ``max_bytes``: largest bf16 payload per call; ``blocks``: workgroups per launch (must be equal on
        every rank — block b of every rank reduces the same range); ``spin_ms``: how long a rank waits for
        a peer before it declares it missing (default ``LWC_AR_SPIN_MS`` or the kernel's ~4 s)."""
        self.group = group
        self.W = dist.get_world_size(group)
        self.me = dist.get_rank(group)
        if self.W > 8:
            raise ValueError("CustomAllReduce supports up to 8 ranks (one xGMI hop)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.cap = (int(max_bytes) + 4095) // 4096 * 4096
        self.blocks = int(blocks)
        k = ops.kernels()
        with torch.cuda.device(self.device):
            self._own, handle = k.ar_alloc(k.ar_region_bytes(self.W, self.cap))
        handles: List[Optional[bytes]] = [None] * self.W
        dist.all_gather_object(handles, handle, group=group)
        self._mapped: List[int] = []
        bases = []
        with torch.cuda.device(self.device):
            for r, h in enumerate(handles):
                if r == self.me:
                    bases.append(self._own)
                else:
                    p = k.ar_open(h)
                    self._mapped.append(p)
                    bases.append(p)
        self.bases = bases
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        if spin_ms is None and os.environ.get("LWC_AR_SPIN_MS"):
            spin_ms = float(os.environ["LWC_AR_SPIN_MS"])
        self.spin_limit = 0 if spin_ms is None else max(1, int(spin_ms * 1e6 / _NS_PER_SPIN))
        # asynchronous error readback: two pinned words (alternating steps) + the event after each copy
        self._err_host = torch.zeros(2, dtype=torch.int32, pin_memory=self.device.type == "cuda")
        self._err_ev: List[Optional[torch.cuda.Event]] = [None, None]
        self._arm_no = 0
        if dist.get_backend(group) == "nccl":
            dist.barrier(group=group, device_ids=[self.device.index])
        else:
            dist.barrier(group=group)
        if self_test is None:
            self_test = os.environ.get("LWC_AR_SELFTEST", "1") != "0"
        if self_test and self.W > 1:
            self.self_test()

    # ------------------------------------------------------------------ start-up self-test
    def _pg_on_device(self) -> bool:
        """Whether the process group's collectives take device tensors (RCCL) rather than host ones (gloo)."""
        return dist.get_backend(self.group) == "nccl"

    def _gather_ref(self, x: torch.Tensor) -> List[torch.Tensor]:
        """Every rank's ``x`` through the process group (host copies; any backend).  ``x`` is built on the
        host: RCCL (backend "nccl") takes device tensors only, gloo host tensors."""
        src = x.to(self.device) if self._pg_on_device() else x.cpu()
        parts = [torch.empty_like(src) for _ in range(self.W)]
        dist.all_gather(parts, src, group=self.group)
        return [p.cpu() for p in parts]

    def self_test(self, numel: int = 1 << 16) -> None:
        """One IPC all-reduce of a random bf16 tensor vs the fp32 sum of the process group's all-gather of the
        same inputs (collective).  Raises :class:`CommFailure` on a mismatch or a raised error word."""
        g = torch.Generator().manual_seed(1234 + self.me)
        x = (torch.rand(numel, generator=g) * 2 - 1).to(torch.bfloat16)
        ref = torch.stack([p.float() for p in self._gather_ref(x)]).sum(0)
        y = x.to(self.device)
        with torch.cuda.device(self.device):
            self.all_reduce_(y)
            torch.cuda.synchronize(self.device)
        got = y.float().cpu()
        bad = int(self.err.item()) != 0 or not torch.allclose(got, ref, atol=0.02 * self.W, rtol=1e-2)
        flag = torch.tensor([1 if bad else 0], dtype=torch.int32)
        dist.all_reduce(flag if dist.get_backend(self.group) != "nccl" else flag.to(self.device),
                        op=dist.ReduceOp.MAX, group=self.group)
        if bad or int(flag.item()):
            raise CommFailure(f"{type(self).__name__} self-test failed on rank {self.me} (max error "
                              f"{(got - ref).abs().max().item():.3g}, error word {int(self.err.item())}): the "
                              "IPC peer mapping does not deliver the peers' data")

    def all_reduce_(self, x: torch.Tensor) -> torch.Tensor:
        """In-place sum of a bf16 tensor over the group (one kernel launch, graph-capturable)."""
        if self.W == 1:
            return x
        if x.dtype != torch.bfloat16 or not x.is_contiguous() or x.numel() % 8:
            raise ValueError("CustomAllReduce: contiguous bf16 tensors of a multiple of 8 elements only")
        k = ops.kernels()
        flat = x.view(-1)
        step = self.cap // 2
        for a in range(0, flat.numel(), step):  # payloads beyond one slot (large prefills): in slot-sized pieces
            piece = flat[a:a + step]
            k.allreduce(self.bases, self.me, piece, piece, self.cap, self.err, self.blocks, self.spin_limit)
        return x

    def arm(self) -> None:
        """Queue an asynchronous copy of the error word behind the work queued so far (call after each
        decode step's launch, outside graph capture); :meth:`poll` reads it later without a sync."""
        if self.W == 1:
            return
        i = self._arm_no & 1
        self._arm_no += 1
        self._err_host[i:i + 1].copy_(self.err, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._err_ev[i] = ev

    def poll(self) -> None:
        """Raise :class:`CommFailure` if an armed copy that has completed shows a failed call (never
        blocks: a copy still in flight is read by a later poll)."""
        for i in (0, 1):
            ev = self._err_ev[i]
            if ev is not None and ev.query():
                self._err_ev[i] = None
                if int(self._err_host[i]):
                    raise CommFailure("CustomAllReduce: a tensor-parallel peer never arrived (spin bound "
                                      "exceeded); the step's activations were poisoned with NaN")

    def check(self) -> None:
        """Raise if any call so far timed out waiting for a peer (host sync; not for the hot path)."""
        if int(self.err.item()):
            raise CommFailure("CustomAllReduce: a peer never arrived (spin timeout)")

    def close(self) -> None:
        k = ops.kernels()
        torch.cuda.synchronize(self.device)
        for p in self._mapped:
            k.ar_close(p)
        self._mapped = []
        if self._own:
            k.ar_free(self._own)
            self._own = 0


class CustomAllToAll(CustomAllReduce):
    """C4: equal-split all-to-all over the same IPC regions and epoch-flag protocol (csrc/kernels/allreduce.hip
    ``alltoall_kernel``): chunk q of this rank's send buffer is stored straight into rank q's region over
    xGMI, and chunk p of the receive buffer is copied out of this rank's region once rank p's flag arrives.
    One launch per exchange, no host synchronisation, graph-capturable — the expert-parallel MoE layer's
    dispatch and combine (parallel/expert.py, padded mode) inside a captured decode step.  ``max_bytes`` is
    the largest per-(source, destination) chunk.  A peer that never arrives poisons the received chunks
    (all-ones bytes: NaN for float payloads) and sets the error word read by :meth:`poll` / :meth:`check`."""

    def self_test(self, rows: int = 64) -> None:
        """One IPC all-to-all of random rows vs the chunks taken from the process group's all-gather of every
        rank's input (collective); raises :class:`CommFailure` on any difference (bytes must match exactly)."""
        g = torch.Generator().manual_seed(4321 + self.me)
        x = torch.randint(-(1 << 30), 1 << 30, (self.W * rows, 4), generator=g, dtype=torch.int32)  # (gloo: no int16)
        parts = self._gather_ref(x)
        ref = torch.cat([parts[p][self.me * rows:(self.me + 1) * rows] for p in range(self.W)])
        out = torch.empty_like(x, device=self.device)
        with torch.cuda.device(self.device):
            self.all_to_all(out, x.to(self.device))
            torch.cuda.synchronize(self.device)
        bad = int(self.err.item()) != 0 or not torch.equal(out.cpu(), ref)
        flag = torch.tensor([1 if bad else 0], dtype=torch.int32)
        dist.all_reduce(flag if dist.get_backend(self.group) != "nccl" else flag.to(self.device),
                        op=dist.ReduceOp.MAX, group=self.group)
        if bad or int(flag.item()):
            raise CommFailure(f"CustomAllToAll self-test failed on rank {self.me} (error word "
                              f"{int(self.err.item())}): the IPC peer mapping does not deliver the peers' chunks")

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """out[p] = rank p's inp chunk for this rank; ``inp`` / ``out``: contiguous, dim 0 = W * rows (any
        dtype; chunks are moved as bytes, padded to 16-byte multiples)."""
        if out.shape != inp.shape or out.dtype != inp.dtype or not out.is_contiguous():
            raise ValueError("CustomAllToAll: out must be a contiguous tensor matching inp")
        if self.W == 1:
            return out.copy_(inp)
        if inp.numel() == 0:
            return out
        src = inp.contiguous().view(-1).view(torch.uint8).view(self.W, -1)
        chunk = src.shape[1]
        cp = (chunk + 15) // 16 * 16
        if cp > self.cap:
            raise ValueError(f"CustomAllToAll: chunk of {chunk} bytes exceeds the {self.cap}-byte slot")
        k = ops.kernels()
        direct = cp == chunk
        if cp != chunk:
            send = torch.zeros(self.W, cp, dtype=torch.uint8, device=inp.device)
            send[:, :chunk].copy_(src)
        else:
            send = src
        recv = out.view(-1).view(torch.uint8).view(self.W, -1) if direct else torch.empty_like(send)
        k.alltoall(self.bases, self.me, send, recv, self.cap, self.err, self.blocks, self.spin_limit)
        if not direct:
            out.view(-1).view(torch.uint8).view(self.W, -1).copy_(recv[:, :chunk])
        return out

