"""Batched voter tally for concurrent score requests.

The reference tallies each request on its own (src/score/completions/client.rs:384-455):
``cw = Vᵀ w``, ``confidence = cw / Σ cw``, voter agreement ``a_l = V_l · confidence``.  One request is
~L x C <= 128 x 20 multiply-adds, so a single tally stays in the C++ consensus core.  Under load many
requests finish their voters in the same event-loop turn; ``TallyBatcher`` collects the tallies
submitted during one turn and, when there are at least ``min_batch`` of them, runs all of them in ONE
launch of the ``vote_tally`` HIP kernel (csrc/kernels/consensus.hip: a workgroup per request, fp64 in the
host's summation order, so the results are bitwise equal to the C++ tally).  Smaller batches, and hosts
without the GPU kernel, take the C++ path.
"""
from __future__ import annotations

import asyncio
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from .. import _runtime as RT


@dataclass
class Tally:
    """The fields of the C++ ``TallyResult`` the orchestrator reads."""

    choice_weight: List[float]
    confidence: List[float]
    voter_confidence: List[float]


def vote_rows(voter_choices):
    """(votes, weights) of a request's voter choices in order; an errored voter has an empty vote."""
    votes = [list(ch.delta.vote) if ch.delta.vote is not None else [] for ch in voter_choices]
    wts = [ch.weight if ch.weight is not None else 0.0 for ch in voter_choices]
    return votes, wts


def _check(votes, weights, C: int) -> None:
    # the host tally's contract (consensus_core.cpp tally)
    if len(votes) != len(weights):
        raise ValueError("tally: votes/weights length mismatch")
    for v in votes:
        if v and len(v) != C:
            raise ValueError("tally: vote length != choices")


def tally_many_gpu(items: Sequence, device, stream=None) -> List[Tally]:
    """K10b over ``items`` = [(votes, weights, C)] in one launch: rows are padded to the largest voter
    count and choice count (padded voters are invalid, padded choices have zero votes).  ``stream``: a
    side stream (the serving path's: the read-back then never waits behind engine work queued on the
    device's default stream)."""
    import torch

    if stream is not None:
        with torch.cuda.stream(stream):
            return tally_many_gpu(items, device)
    from .. import ops

    for votes, wts, C in items:
        _check(votes, wts, C)
    R = len(items)
    L = max(1, max(len(v) for v, _, _ in items))
    Cm = max(C for _, _, C in items)
    V = np.zeros((R, L, Cm), dtype=np.float64)
    W = np.zeros((R, L), dtype=np.float64)
    ok = np.zeros((R, L), dtype=np.uint8)
    for r, (votes, wts, C) in enumerate(items):
        for l, v in enumerate(votes):
            W[r, l] = wts[l]
            if v:
                V[r, l, :C] = v
                ok[r, l] = 1
    cw, conf, vconf = ops.vote_tally(torch.from_numpy(V).to(device), torch.from_numpy(W).to(device),
                                     torch.from_numpy(ok).to(device))
    cw, conf, vconf = cw.cpu().numpy(), conf.cpu().numpy(), vconf.cpu().numpy()
    out = []
    for r, (votes, _, C) in enumerate(items):
        out.append(Tally(cw[r, :C].tolist(), conf[r, :C].tolist(), vconf[r, :len(votes)].tolist()))
    return out


class TallyBatcher:
    """Collects the tallies requested during one event-loop turn; ``min_batch`` or more run as one K10b
    launch on ``device`` (launched and read back on a worker thread), fewer on the host C++ tally.
    ``device=None`` keeps everything on the host.  Each item is validated on its own first: a malformed
    vote fails only its request."""

    def __init__(self, device=None, min_batch: int = 8):
        self.device = device
        self.min_batch = max(1, int(min_batch))
        self._pending: list = []
        self._scheduled = False
        self.gpu_batches = 0  # launches so far (observability / tests)
        self.gpu_tallies = 0
        self._stream = None  # created on the first GPU batch (a non-blocking side stream)
        self._sched_loop = None
        self._executor = None  # one worker thread: GPU batches launch and read back off the event loop

    async def tally(self, voter_choices, C_len: int):
        votes, wts = vote_rows(voter_choices)
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._pending.append((votes, wts, C_len, fut))
        if not self._scheduled or self._sched_loop is not loop:
            # (a flush scheduled on a loop that has since closed never runs: schedule on this one)
            self._scheduled, self._sched_loop = True, loop
            loop.call_soon(self._flush)
        return await fut

    def _flush(self) -> None:
        batch, self._pending, self._scheduled = self._pending, [], False
        # skip cancelled futures and those of an event loop that has closed (nobody can await them)
        live = [b for b in batch if not b[3].done() and not b[3].get_loop().is_closed()]
        good = []
        for item in live:  # a malformed vote fails its own request only (as the host tally would)
            try:
                _check(item[0], item[1], item[2])
                good.append(item)
            except ValueError as e:
                item[3].set_exception(e)
        if not good:
            return
        if self.device is not None and len(good) >= self.min_batch:
            # the launch and its read-back run on a worker thread: the event loop never blocks on a device
            # sync (it keeps streaming other requests' chunks while the batch is on the GPU)
            loop = good[0][3].get_loop()
            if self._executor is None:
                from concurrent.futures import ThreadPoolExecutor

                self._executor = ThreadPoolExecutor(max_workers=1, thread_name_prefix="k10b")
            fut = loop.run_in_executor(self._executor, self._gpu_batch, [(v, w, c) for v, w, c, _ in good])
            fut.add_done_callback(lambda f, good=good: self._deliver(good, f))
            return
        self._host(good)

    def _gpu_batch(self, items):
        import contextlib

        import torch

        on_cuda = str(self.device).startswith("cuda")
        with torch.cuda.device(torch.device(self.device)) if on_cuda else contextlib.nullcontext():
            if self._stream is None:
                self._stream = torch.cuda.Stream(device=self.device)
            return tally_many_gpu(items, self.device, self._stream)

    def _deliver(self, good, f) -> None:
        try:
            res = f.result()
        except Exception:  # noqa: BLE001 — a device error must not strand the awaiting requests:
            self._host(good)  # they fall back to the host tally
            return
        self.gpu_batches += 1
        self.gpu_tallies += len(good)
        for (_, _, _, fut), t in zip(good, res):
            if not fut.done():
                fut.set_result(t)

    @staticmethod
    def _host(items) -> None:
        for votes, wts, C, fut in items:
            if fut.done():
                continue
            try:
                fut.set_result(RT.tally(votes, wts, C))
            except Exception as e:  # noqa: BLE001 — surfaced to the awaiting request
                fut.set_exception(e)


def make_batcher(spec: Optional[str], device) -> Optional[TallyBatcher]:
    """``LWC_GPU_TALLY``: unset / "0" = host tally per request; N >= 1 = batch concurrent tallies and run
    batches of at least N requests on the GPU."""
    if not spec or spec.strip() in ("0", "off", "false"):
        return None
    return TallyBatcher(device, int(spec))
