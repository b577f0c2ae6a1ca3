"""Continuous-batching generation engine for one MI355X (one process per GPU).

This is the in-process replacement of the reference's upstream-provider round trip
(src/chat/completions/client.rs:193-434): a request becomes a *sequence group* of n sequences that
share their prompt's KV blocks (prefill once, fork n times — the multichat/voter fan-out of
src/score/completions/client.rs:343-356 mapped onto one GPU), and every `step()` advances all running
sequences by one token with a single batched decode launch.

Host runtime pieces are native C++ (`_runtime.BlockManager`: ref-counted paged-KV blocks with
copy-on-write fork, `prepare_decode_into`: per-step batch tables written straight into pinned staging).  The decode forward is captured once per
batch bucket into a hipGraph (torch.cuda.CUDAGraph on ROCm) so a step is one graph replay plus the
fused sampler launch.

KV admission and over-subscription: a group is admitted against a RESERVATION of its prompt blocks plus
``kv_reserve_tokens`` of growth per sequence (not n * max_tokens: a voter passing a large ``max_tokens``
through, reference src/score/llm/mod.rs:44,56, would otherwise throttle the whole GPU), and the physical
pool must hold the prompt plus one block per sequence above a watermark.  Sequences that grow past their
reservation take blocks from the pool; when a decode step would need more blocks than are free, the
YOUNGEST running groups are preempted by SWAPPING: their distinct KV blocks (the shared prompt blocks
once) are copied to pinned host memory in stream order and the blocks freed; they resume, oldest first
and before any new admission, when the pool can hold them again — KV bytes come back unchanged, so a
preempted request produces exactly the tokens of an uninterrupted run.
"""
from __future__ import annotations

import gc
import itertools
import os
import random
import sys
import threading
import time
from array import array
from collections import deque
from dataclasses import dataclass
from typing import Callable, Deque, Dict, List, Optional, Sequence as Seq, Tuple

import numpy as np
import torch

from .. import ops
from ..utils.faults import FaultInjector
from ..utils.tracing import RequestTimer, span
from .._runtime import BlockManager, prepare_decode_into, slots_range
from ..models.llama import KVCache
from .sampling import SamplingParams
from .tokenizer import IncrementalDecoder

BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128, 256, 384, 512, 768, 1024, 1536, 2048, 3072, 4096, 5120, 6144, 8192)


@dataclass
class TokenEvent:
    seq: "Sequence"
    token_id: int
    text: str
    logprob: float
    top_logprobs: List[Tuple[int, float]]
    finished: bool = False
    finish_reason: Optional[str] = None


class Sequence:
    _ids = itertools.count(1)

    def __init__(self, group: "SequenceGroup", index: int, seed: int):
        self.id = next(Sequence._ids)
        self.group = group
        self.index = index
        self.seed = seed
        self.n_launched = 0  # tokens sampled or in flight (the Philox offset of the next sample)
        # generated ids as a flat int32 array: the encoders pack thousands of them with one zero-copy view
        # per sequence (models/packing.py) instead of converting Python ints
        self.tokens = array("i")
        self._text: Optional[str] = None  # streamed text (callback / stop strings), else decoded on demand
        self.finished = False
        self.finish_reason: Optional[str] = None
        self.count_row = -1
        self.constraint_state = None
        self.detok = IncrementalDecoder(group.engine.tokenizer)

    @property
    def params(self) -> SamplingParams:
        return self.group.params

    @property
    def text(self) -> str:
        """Generated text.  Streamed incrementally when a callback or stop strings need it during
        generation; otherwise decoded from the tokens on first access (no per-token host work)."""
        if self._text is not None:
            return self._text
        tok = self.group.engine.tokenizer
        eos = tok.eos_token_id
        ids = [t for t in self.tokens if t != eos and t not in self.params.stop_token_ids]
        return tok.decode(ids)

    @text.setter
    def text(self, v: str) -> None:
        self._text = v


class SequenceGroup:
    _ids = itertools.count(1)

    def __init__(self, engine: "LLMEngine", prompt_ids: List[int], params: SamplingParams, n: int,
                 callback: Optional[Callable[[TokenEvent], None]]):
        self.id = next(SequenceGroup._ids)
        self._chain: Optional[List[int]] = None  # chained block hashes of the prompt (LLMEngine._block_chain)
        self.engine = engine
        self.prompt_ids = list(prompt_ids)
        self.params = params
        self.n = n
        self.callback = callback
        base = params.seed if params.seed is not None else random.getrandbits(63)
        off = params.seed_offset
        self.seqs = [Sequence(self, i, (base * 1000003 + off + i) & ((1 << 63) - 1)) for i in range(n)]
        self.bias_row = -1
        self.reserved_blocks = 0
        self.timer = RequestTimer()
        self.prefilled: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
        self.pf_pos = -1  # chunked prefill: prompt tokens already in the KV cache (-1 = not started)
        # request context (context.RequestContext): admission priority, deadline, trace id
        self.priority = 0
        self.deadline: Optional[float] = None
        self.trace_id: Optional[str] = None

    @property
    def finished(self) -> bool:
        return all(s.finished for s in self.seqs)


_F32_PARAMS = ("temperature", "top_p", "min_p", "top_a", "freq_pen", "pres_pen", "rep_pen")
_I32_PARAMS = ("top_k", "count_rows", "bias_rows")


class _GraphBucket:
    """Per batch-size bucket: the captured decode graph plus ONE int32 staging layout holding every
    per-step input (block tables, ctx lens, slots, positions, tokens, prefix tiles, sampler
    parameters, Philox seeds/offsets).  The host side is two pinned buffers (alternating steps), the
    device side one buffer whose views are the graph's inputs, so a step is one H2D copy."""

    def __init__(self, B: int, width: int, splits: int, max_tiles: int, device):
        self.B, self.width, self.splits, self.max_tiles = B, width, splits, max_tiles
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.logits: Optional[torch.Tensor] = None
        # captured decode graphs by attention mode (True = cascade, False = plain split-K), sharing one
        # memory pool, and their output logits
        self.graphs: Dict[bool, torch.cuda.CUDAGraph] = {}
        self.graph_logits: Dict[bool, torch.Tensor] = {}
        self.pool = None
        segs: List[Tuple[str, int]] = [("block_tables", B * width), ("ctx_lens", B), ("slots", B), ("positions", B),
                                       ("tokens", B), ("tiles", max(1, max_tiles) * 3)]
        segs += [(n, B) for n in _F32_PARAMS + _I32_PARAMS]
        segs += [("seeds", 2 * B), ("offsets", 2 * B)]
        self.off: Dict[str, Tuple[int, int]] = {}
        o = 0
        for name, n in segs:
            o += o & 1  # keep every segment 8-byte aligned (int64 views)
            self.off[name] = (o, o + n)
            o += n
        self.size = o + (o & 1)
        self.dev = torch.zeros(self.size, dtype=torch.int32, device=device)
        self.host = [torch.zeros(self.size, dtype=torch.int32).pin_memory() for _ in range(2)]
        self.host_static_key: List[object] = [None, None]
        self.d = self._views(self.dev, torch)
        self.h = [self._views(h.numpy(), np) for h in self.host]
        self.out_dev: List[Optional[torch.Tensor]] = [None, None]
        self.out_host: List[Optional[torch.Tensor]] = [None, None]

    def _views(self, buf, lib):
        f32 = torch.float32 if lib is torch else np.float32
        i64 = torch.int64 if lib is torch else np.int64
        v = {}
        for name, (a, b) in self.off.items():
            x = buf[a:b]
            if name in _F32_PARAMS:
                x = x.view(f32)
            elif name in ("seeds", "offsets"):
                x = x.view(i64)
            v[name] = x
        v["block_tables"] = v["block_tables"].reshape(self.B, self.width)
        v["tiles"] = v["tiles"].reshape(max(1, self.max_tiles), 3)
        return v

    def outputs(self, parity: int, K: int):
        """Sampler outputs for one step as views of one device buffer (tok | lp | topk ids | topk lp),
        and the matching pinned host buffer (one D2H copy per step)."""
        B, Kb = self.B, max(K, 1)
        need = B * (2 + 2 * Kb)
        if self.out_dev[parity] is None or self.out_dev[parity].numel() < need:
            self.out_dev[parity] = torch.empty(need, dtype=torch.int32, device=self.dev.device)
            self.out_host[parity] = torch.empty(need, dtype=torch.int32).pin_memory()
        o = self.out_dev[parity]
        tok = o[:B]
        lp = o[B:2 * B].view(torch.float32)
        ids = o[2 * B:2 * B + B * Kb].view(B, Kb)
        lps = o[2 * B + B * Kb:need].view(torch.float32).view(B, Kb)
        return (tok, lp, ids, lps), o[:need], self.out_host[parity][:need]


def cascade_table_size(B: int, per_tile: int) -> int:
    """Rows of a bucket's cascade tile table: one tile per `per_tile` sequences plus slack for group
    boundaries — enough for every group to own a tile down to groups of 8 sequences (e.g. 64 candidates
    split over 8 GPUs); smaller groups beyond the slack degrade to plain rows (:func:`cascade_tiles`).
    Unused entries are workgroups that exit at once (measured: no cost vs an exact grid)."""
    return -(-B // per_tile) + B // 8 + 1


def cascade_tiles(runs: List[Tuple[int, int, int]], per_tile: int, tiles: np.ndarray) -> int:
    """Fill `tiles` [T, 3] with cascade super-tiles (row_start, nseq, prefix_blocks).

    `runs` are the batch's consecutive (start, count, prompt_blocks) sequence runs, one per group.
    Runs of >= 2 sequences with a non-empty prompt block prefix get their own tiles (<= per_tile
    sequences each); everything else is packed into plain tiles (prefix_blocks = 0).  If the table
    would overflow, the remaining groups degrade to plain rows.  Returns the number of tiles."""
    T = tiles.shape[0]
    tiles[:] = 0
    nt = 0
    plain: List[int] = []  # [start, end) of the pending plain stretch

    def emit(r0: int, n: int, pblk: int):
        nonlocal nt
        for a in range(r0, r0 + n, per_tile):
            if nt >= T:
                raise RuntimeError("cascade plan: tile table overflow")
            tiles[nt] = (a, min(per_tile, r0 + n - a), pblk)
            nt += 1

    def flush():
        if plain:
            emit(plain[0], plain[1] - plain[0], 0)
            plain.clear()

    total = sum(n for _, n, _ in runs)
    for idx, (start, n, pblk) in enumerate(runs):
        shared = n >= 2 and pblk > 0
        if shared:
            # tiles this run needs + a worst-case plain tail must still fit
            rest = total - (start + n)
            pending = -(-(plain[1] - plain[0]) // per_tile) if plain else 0
            need = pending + -(-n // per_tile) + -(-rest // per_tile)
            if nt + need > T:
                shared = False
        if shared:
            flush()
            emit(start, n, pblk)
        else:
            if plain and plain[1] == start:
                plain[1] = start + n
            else:
                flush()
                plain.extend([start, start + n])
    flush()
    return nt


class _PinnedRing:
    """Pinned host staging for the engine's per-step uploads: one pinned arena used as a ring.  An upload
    copies into the next free region and issues a non-blocking copy from it; a region is written again only
    after the event recorded behind its upload completed (oldest first, the ring's own order).  A fresh
    ``pin_memory()`` per upload cost ~250 us of host time each (~15 per mixed step; serve_load cProfile)."""

    def __init__(self, nbytes: int = 32 << 20):
        self.buf = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self.n, self.head = nbytes, 0
        self.live: Deque[Tuple[int, int, "torch.cuda.Event"]] = deque()

    def upload(self, t: torch.Tensor, dev) -> torch.Tensor:
        nb = t.numel() * t.element_size()
        size = (nb + 255) & ~255
        if size > self.n // 4:
            return t.pin_memory().to(dev, non_blocking=True)
        if self.head + size > self.n:
            self.head = 0
        start, end = self.head, self.head + size
        while self.live and self.live[0][0] < end and start < self.live[0][1]:
            self.live.popleft()[2].synchronize()  # (regions are handed out in order: the oldest overlaps first)
        self.head = end
        dst = self.buf[start:start + nb].view(t.dtype).view(t.shape)
        dst.copy_(t)
        out = dst.to(dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.live.append((start, end, ev))
        if len(self.live) > 4096:  # bounded bookkeeping: retire the oldest
            self.live.popleft()[2].synchronize()
        return out


_RINGS = threading.local()


def _h2d(x, dtype, dev) -> torch.Tensor:
    """Host list / array -> device through pinned memory, non-blocking: a pageable upload synchronises
    the stream, i.e. would hold the host until every queued kernel (a decode step in flight) finished.
    Staged through this thread's pinned ring (one per engine thread and device)."""
    t = (torch.from_numpy(np.ascontiguousarray(x)) if isinstance(x, np.ndarray) else torch.tensor(x)).to(dtype)
    dev = torch.device(dev)
    if dev.type != "cuda":
        return t.to(dev)
    rings = getattr(_RINGS, "by_dev", None)
    if rings is None:
        rings = _RINGS.by_dev = {}
    ring = rings.get(dev)
    if ring is None:
        ring = rings[dev] = _PinnedRing()
    return ring.upload(t.contiguous(), dev)


class _Step:
    """A launched (not yet processed) decode step."""

    def __init__(self, seqs, key, bk, parity, K, tok_dev, out_host, event):
        self.seqs, self.key, self.bk, self.parity, self.K = seqs, key, bk, parity, K
        self.tok_dev, self.out_host, self.event = tok_dev, out_host, event
        self.static = None  # the launch's static sampler inputs (deferred sampler launch)
        self.first = None   # first-token step after a prefill: (pinned host outputs, groups)


@dataclass
class _SwapRecord:
    """A preempted group: its live sequences' KV (distinct blocks) in pinned host memory."""
    group: "SequenceGroup"
    seqs: List[Sequence]
    host: torch.Tensor          # [L, 2, n, block_elems] pinned
    tables: List[List[int]]     # per sequence: indices into the n saved blocks
    lens: List[int]
    event: Optional[torch.cuda.Event]


class LLMEngine:
    def __init__(self, model, tokenizer, *, block_size: int = 16, num_blocks: Optional[int] = None,
                 kv_memory_fraction: float = 0.85, max_batch: int = 512, max_model_len: int = 4096,
                 use_graphs: bool = True, prefill_token_budget: int = 16384, prefix_sharing: bool = True,
                 cascade_min_batch: int = 128, tune_gc: bool = True, constrained_logprobs: bool = False,
                 prefix_caching: bool = False, chunked_prefill: int = 0, kv_reserve_tokens: Optional[int] = 256,
                 decode_splits: Optional[int] = None):
        self.model = model
        self.cfg = model.cfg
        self.tokenizer = tokenizer
        self.device = model.device
        self.block_size = block_size
        self.max_batch = max_batch
        self.max_model_len = max_model_len
        self.prefill_token_budget = prefill_token_budget
        # chunked prefill (serving): admitted prompts are prefilled at most `chunked_prefill` tokens per
        # engine step, in the same forward as that step's decode rows, so running sequences never stall
        # behind an admission (0 = whole admission batches, then decode: the throughput bench's mode)
        self.chunked_prefill = int(chunked_prefill)
        self._mixed_tuned = False
        if self.chunked_prefill and self.cfg.head_dim != 128:
            raise ValueError("chunked prefill: the paged-KV prefill kernel is built for head_dim 128")
        self.prefilling: List[SequenceGroup] = []
        self.width = (max_model_len + block_size - 1) // block_size
        if num_blocks is None:
            free, _total = torch.cuda.mem_get_info(self.device)
            per = KVCache.bytes_per_block(self.cfg, block_size)
            num_blocks = max(64, int(free * kv_memory_fraction) // per)
        self.cache = KVCache(self.cfg, num_blocks, block_size, self.device)
        self.bm = BlockManager(num_blocks, block_size)
        # cross-request prefix cache (C++ block manager): prompts that start with an already computed
        # token prefix (the shared messages of a score request's voters, a repeated conversation) reuse
        # its full KV blocks and prefill only the tail
        self.prefix_caching = prefix_caching
        self.bm.set_prefix_caching(prefix_caching)
        self.free_blocks_unreserved = num_blocks
        # growth reserved per sequence at admission (None: worst case, prompt + max_tokens — no preemption)
        self.kv_reserve_tokens = kv_reserve_tokens
        self.kv_watermark = max(1, num_blocks // 100)
        self.swapped: Deque[_SwapRecord] = deque()
        # split-K factor of the plain paged-decode kernel (None: chosen per batch bucket)
        self.decode_splits = decode_splits
        self.use_graphs = use_graphs
        self.prefix_sharing = prefix_sharing
        # decode batches >= this bucket use the cascade (shared-prompt) attention kernel; smaller ones
        # the split-K kernel, which spreads a few long contexts over more workgroups
        self.cascade_min_batch = cascade_min_batch
        # report logprobs of grammar-constrained steps over the allowed tokens only (vote fast path:
        # at a constrained key letter that is the restricted softmax over the sibling letters)
        self.constrained_logprobs = constrained_logprobs
        self.buckets: Dict[int, _GraphBucket] = {}
        self.step_ab: Dict[int, dict] = {}  # bucket -> in-step A/B replay times per plan (_step_ab)
        self.inflight: Optional[_Step] = None
        # first tokens after a prefill are sampled asynchronously and processed by the next decode step
        self.async_first_tokens = True
        self._step_no = 0
        self._comp_cache: Tuple[object, Optional[dict]] = (None, None)
        self.waiting: Deque[SequenceGroup] = deque()
        self.running: List[Sequence] = []
        self.lock = threading.Lock()
        V = self.cfg.vocab_size
        self.counts: Optional[torch.Tensor] = None  # [max_batch, V] int16, lazily
        self.free_count_rows = list(range(max_batch))
        self.bias: Optional[torch.Tensor] = None    # [max_batch, V] f32, lazily
        self.free_bias_rows = list(range(max_batch))
        self.stats = {"prefill_tokens": 0, "decode_tokens": 0, "steps": 0, "prefix_cache_tokens": 0,
                      "preemptions": 0, "swapped_blocks": 0}
        self._mask_rows_of: Optional[Dict[tuple, int]] = None  # mask content -> device mask table row
        self._mask_limit = 4096
        self.faults = FaultInjector.from_env()
        self._deadlines = 0  # groups ever submitted with a deadline (expire() is a no-op until one is)
        # step() returns TokenEvents only when asked (callbacks always get theirs)
        self.collect_events = False
        if tune_gc:
            # thousands of live sequences make full collections (triggered by the per-token
            # allocation churn) cost ~100 ms pauses that stall the GPU; raise the gen-0 threshold
            gc.set_threshold(max(gc.get_threshold()[0], 200_000), 50, 100)

    # ------------------------------------------------------------------ API
    def add_request(self, prompt_ids: Seq[int], params: SamplingParams, n: int = 1,
                    callback: Optional[Callable[[TokenEvent], None]] = None,
                    prefilled: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, ctx=None) -> SequenceGroup:
        """Queue a request of `n` sequences.  ``prefilled`` = (kv [L, 2, nblocks, block_elems],
        logits [V]) starts it from a prompt prefilled elsewhere (see :meth:`export_prefill`).  ``ctx`` (a
        context.RequestContext or a dict with ``priority`` / ``deadline`` / ``trace_id``): requests are
        admitted by priority (higher first, FIFO within one) and dropped once their deadline passes
        (:meth:`expire`)."""
        params.validate(self.cfg.vocab_size)
        if params.constraint is not None and hasattr(params.constraint, "bind"):
            params.constraint.bind(self.tokenizer, self.cfg.vocab_size)  # a constraint that came through a pipe
        if len(prompt_ids) == 0:
            raise ValueError("empty prompt")
        if len(prompt_ids) + params.max_tokens > self.max_model_len:
            raise ValueError(f"prompt ({len(prompt_ids)}) + max_tokens ({params.max_tokens}) exceeds "
                             f"max_model_len ({self.max_model_len})")
        g = SequenceGroup(self, list(prompt_ids), params, n, callback)
        g.prefilled = prefilled
        if isinstance(ctx, dict):
            g.priority = int(ctx.get("priority", 0) or 0)
            g.deadline = ctx.get("deadline")
            g.trace_id = ctx.get("trace_id")
            g.timer.trace_id = g.trace_id
        with self.lock:
            if g.priority and self.waiting and self.waiting[-1].priority < g.priority:
                # ahead of every waiting request of lower priority, behind its own priority's
                i = next(k for k, x in enumerate(self.waiting) if x.priority < g.priority)
                self.waiting.insert(i, g)
            else:
                self.waiting.append(g)
            if g.deadline is not None:
                self._deadlines += 1
        return g

    def has_work(self) -> bool:
        return (bool(self.waiting) or bool(self.running) or bool(self.prefilling) or bool(self.swapped)
                or self.inflight is not None)

    def step(self) -> List[TokenEvent]:
        """Run one engine iteration: admit+prefill waiting groups if any fit, else one decode step.

        Decode steps are pipelined one deep: step t+1 is launched (its inputs need only the block
        manager, and its input tokens are step t's sampler output, still on the device) BEFORE the
        host syncs on and post-processes step t, so detokenisation, stop checks and callbacks overlap
        the GPU.  A sequence that finishes at step t has one discarded row in step t+1."""
        self.faults.on_step()
        if self.swapped:
            self._swap_in()
        if self.chunked_prefill > 0:
            return self._step_chunked()
        events: List[TokenEvent] = []
        with self.lock:
            fits = self._first_waiting_fits()
        if fits:
            events += self._drain()
            with span("schedule"), self.lock:
                admitted = self._admit()
            if admitted:
                with span("prefill"):
                    return events + self._prefill(admitted)
        if self.running or self.inflight is not None:
            events += self._decode()
        return events

    def generate(self, prompts: List[List[int]], params: SamplingParams, n: int = 1) -> List[List[List[int]]]:
        """Offline helper: run prompts to completion, return tokens[prompt][choice]."""
        groups = [self.add_request(p, params, n) for p in prompts]
        while self.has_work():
            self.step()
        return [[list(s.tokens) for s in g.seqs] for g in groups]

    # ------------------------------------------------------------------ scheduling
    def _group_reservation(self, g: SequenceGroup) -> int:
        bs = self.block_size
        prompt_blocks = (len(g.prompt_ids) + bs - 1) // bs
        grow = g.params.max_tokens if self.kv_reserve_tokens is None else min(g.params.max_tokens,
                                                                               self.kv_reserve_tokens)
        per_child = (len(g.prompt_ids) + grow + bs - 1) // bs - len(g.prompt_ids) // bs
        return prompt_blocks + g.n * (per_child + 1)

    def _physical_need(self, g: SequenceGroup) -> int:
        """Blocks the pool must have free to admit ``g``: its prompt, one growth block per sequence and the
        watermark (sequences past their reservation draw on the same pool)."""
        return (len(g.prompt_ids) + self.block_size - 1) // self.block_size + g.n + self.kv_watermark

    def _first_waiting_fits(self) -> bool:
        if not self.waiting or self.swapped:  # preempted groups resume before anything new is admitted
            return False
        g = self.waiting[0]
        live = sum(1 for s in self.running if not s.finished) + sum(x.n for x in self.prefilling)
        idle = not self.running and self.inflight is None and not self.prefilling
        return live + g.n <= self.max_batch and ((self._group_reservation(g) <= self.free_blocks_unreserved
                                                  and self._physical_need(g) <= self.bm.num_free) or idle)

    def _admit(self) -> List[SequenceGroup]:
        out, tokens = [], 0
        while self.waiting:
            g = self.waiting[0]
            need = self._group_reservation(g)
            if len(self.running) + sum(x.n for x in self.prefilling) + sum(x.n for x in out) + g.n > self.max_batch:
                break
            phys = self._physical_need(g) + sum(self._physical_need(x) - self.kv_watermark for x in out)
            if need > self.free_blocks_unreserved or phys > self.bm.num_free:
                if not self.running and not out and not self.prefilling:
                    self.waiting.popleft()
                    raise RuntimeError("request needs more KV blocks than the cache holds")
                break
            cost = len(g.prompt_ids) if g.prefilled is None else 0  # imported prompts cost no compute
            if out and tokens + cost > self.prefill_token_budget:
                break
            self.faults.on_admit()
            self.waiting.popleft()
            g.reserved_blocks = need
            g.timer.started()
            self.free_blocks_unreserved -= need
            tokens += cost
            out.append(g)
        return out

    # ------------------------------------------------------------------ prefill
    def _run_prefill(self, prompts: List[List[int]], parents: List[int], use_cache: bool = False) -> torch.Tensor:
        """Prefill packed prompts into freshly added transient sequences `parents`; returns the
        last-token logits [len(prompts), V].  With ``use_cache`` the prompts' cached prefix blocks are
        taken from the prefix cache and only the tails are computed (attention still sees the whole
        prompt), and the prompts' full blocks are registered for later requests."""
        added: List[int] = []
        try:
            return self._run_prefill_inner(prompts, parents, use_cache, added)
        except BaseException:
            # a later prompt of the wave ran out of KV blocks (or the prefill failed): release the transient
            # parents already created and the cached blocks they acquired, then re-raise
            for pid in added:
                self.bm.free_sequence(pid)
            raise

    def _run_prefill_inner(self, prompts, parents, use_cache, added) -> torch.Tensor:
        dev = self.device
        toks, pos, slots, cu, last, cached = [], [], [], [0], [], []
        for pid, p in zip(parents, prompts):
            L = len(p)
            c = int(self.bm.add_sequence_cached(pid, p)) if use_cache else 0
            if not use_cache:
                self.bm.add_sequence(pid, L)
            added.append(pid)
            cached.append(c)
            toks.extend(p[c:])
            pos.extend(range(c, L))
            slots.append(slots_range(self.bm, pid, c, L - c))
            cu.append(cu[-1] + L - c)
            last.append(cu[-1] - 1)
        ctx = None
        if any(cached):
            k_lens = [len(p) for p in prompts]
            ks = np.concatenate([slots_range(self.bm, pid, 0, L) for pid, L in zip(parents, k_lens)]).astype(np.int64)
            if ks.size and (ks.min() < 0 or ks.max() >= self.bm.num_blocks * self.block_size):
                raise RuntimeError("prefix-cache prefill: KV slot out of range")
            ctx = {"k_slots": _h2d(ks, torch.int64, dev),
                   "cu_k": _h2d(np.concatenate([[0], np.cumsum(k_lens)]), torch.int32, dev),
                   "q_lens": [L - c for L, c in zip(k_lens, cached)], "k_lens": k_lens}
            self.stats["prefix_cache_tokens"] += sum(cached)
        t_tok = _h2d(toks, torch.int32, dev)
        t_pos = _h2d(pos, torch.int32, dev)
        t_slots = _h2d(np.concatenate(slots), torch.int32, dev)
        t_cu = _h2d(cu, torch.int32, dev)
        t_last = _h2d(last, torch.int64, dev)
        max_len = max(len(p) - c for p, c in zip(prompts, cached))
        logits = self.model.prefill(t_tok, t_pos, t_slots, t_cu, max_len, t_last, self.cache, ctx=ctx)
        if use_cache:
            for pid, p in zip(parents, prompts):
                self.bm.cache_prefix(pid, p)
        self.stats["prefill_tokens"] += len(toks)
        return logits

    def export_prefill(self, prompts: List[List[int]]) -> Tuple[torch.Tensor, torch.Tensor, List[int]]:
        """Prefill prompts WITHOUT starting any sequences and return what another engine needs to
        start them without recomputing: (kv [L, 2, sum(nblocks), block_elems], logits [n, V], nblocks).

        This is the multi-GPU candidate-parallel path: each rank prefills its own share of the
        requests, the prompt KV blocks and last-token logits are all-gathered over RCCL, and every
        rank then samples its candidates of every request from the imported prompts
        (:meth:`add_request` with ``prefilled=``).  Must be called between steps."""
        if self.inflight is not None:
            raise RuntimeError("export_prefill while a decode step is in flight")
        parents = [-(1 << 40) - i for i in range(len(prompts))]
        need = sum((len(p) + self.block_size - 1) // self.block_size for p in prompts)
        if need > self.free_blocks_unreserved:
            raise RuntimeError("export_prefill: not enough free KV blocks")
        logits = self._run_prefill(prompts, parents)
        blocks: List[int] = []
        nblocks: List[int] = []
        for pid in parents:
            tab = list(self.bm.block_table(pid))
            blocks.extend(tab)
            nblocks.append(len(tab))
        idx = torch.tensor(blocks, dtype=torch.int64, device=self.device)
        kv = self.cache.pool.index_select(2, idx)
        for pid in parents:
            self.bm.free_sequence(pid)
        return kv, logits, nblocks

    def _prefill(self, groups: List[SequenceGroup]) -> List[TokenEvent]:
        dev = self.device
        compute = [g for g in groups if g.prefilled is None]
        imported = [g for g in groups if g.prefilled is not None]
        logits_of: Dict[int, torch.Tensor] = {}
        for wave in self._prefill_waves(compute):
            lg = self._run_prefill([g.prompt_ids for g in wave], [-g.id for g in wave],
                                   use_cache=self.prefix_caching)
            for i, g in enumerate(wave):
                logits_of[g.id] = lg[i]
        for g in imported:
            kv, row = g.prefilled
            parent = -g.id
            self.bm.add_sequence(parent, len(g.prompt_ids))
            tab = torch.tensor(list(self.bm.block_table(parent)), dtype=torch.int64, device=dev)
            if kv.shape[2] != tab.numel():
                raise ValueError(f"imported KV has {kv.shape[2]} blocks, prompt needs {tab.numel()}")
            self.cache.pool.index_copy_(2, tab, kv)
            logits_of[g.id] = row
            g.prefilled = None  # drop the reference: the cache owns the data now
        return self._start_groups(groups, logits_of)

    def _start_groups(self, groups: List[SequenceGroup], logits_of: Dict[int, torch.Tensor]) -> List[TokenEvent]:
        """Fork every prefilled group into its n sequences (shared prompt blocks), sample their first
        tokens from the prompt's last-token logits and add them to the running batch."""
        rows, seqs = [], []
        for g in groups:
            parent = -g.id
            for s in g.seqs:
                self.bm.fork(parent, s.id)
                self._attach_rows(s)
                rows.append(logits_of[g.id])
                seqs.append(s)
            self.bm.free_sequence(parent)
        if self.async_first_tokens and self.inflight is None and self.device.type == "cuda":
            self.inflight = self._launch_first(torch.stack(rows), seqs, groups)
            self.running.extend(seqs)
            return []
        events = self._sample_and_advance(torch.stack(rows), seqs)
        for g in groups:
            g.timer.token()
        for s in seqs:
            if not s.finished:
                self.running.append(s)
        return events

    # ------------------------------------------------------------------ chunked prefill
    def _step_chunked(self) -> List[TokenEvent]:
        """One engine step in chunked-prefill mode.  Admitted prompts are prefilled at most
        ``chunked_prefill`` tokens per step, and a step that has prompt tokens to prefill is ONE forward over
        [every running sequence's next token || the prompt-chunk rows] (:meth:`_mixed_step`): one GEMM per
        projection over both, decode rows on the paged decode kernel, chunk rows on the paged-KV prefill
        kernel — running sequences advance by a token in every step, a long prompt never stalls them.
        Steps with nothing to prefill are the plain (graph-captured) decode step."""
        events: List[TokenEvent] = []
        with self.lock:
            fits = self._first_waiting_fits()
            admitted = self._admit() if fits else []
        self.prefilling.extend(admitted)
        imported = [g for g in self.prefilling if g.prefilled is not None]
        if imported:  # prompts prefilled elsewhere cost no compute: start them now
            events += self._drain()
            self.prefilling = [g for g in self.prefilling if g.prefilled is None]
            events += self._prefill(imported)
        if self.prefilling:
            items, _budget, _deferred = self._chunk_items(self.chunked_prefill)
            if items:
                with span("prefill.mixed"):
                    events += self._mixed_step(items)
                return events
        if self.running or self.inflight is not None:
            events += self._decode()
        return events

    def _mixed_step(self, items: List[Tuple[SequenceGroup, int, int]]) -> List[TokenEvent]:
        """One forward over the decode rows of every running sequence and the prompt-chunk rows of
        ``items`` ((group, a, e): prompt tokens [a, e) of the group's parent sequence); the decode rows'
        next tokens and the first tokens of prompts completed by this chunk are sampled in one launch that
        becomes the in-flight step.

        Pipelined like the decode step: the forward is launched BEFORE the previous step is processed on the
        host (the decode rows of sequences still in that step take their input token from its sampler output
        on the device), the sampler after it (grammar masks need the previous tokens on the host).  A row of a
        sequence that the previous step finishes is computed and discarded."""
        dev = self.device
        events: List[TokenEvent] = []
        if not self._mixed_tuned:
            self._tune_mixed()
        prev, self.inflight = self.inflight, None
        self.running = [s for s in self.running if not s.finished]
        dec = [s for s in self.running if s.n_launched < s.params.max_tokens]
        if dec and self.bm.append_cost_total([s.id for s in dec]) > self.bm.num_free:
            if prev is not None:  # preemption swaps KV out: nothing may be in flight
                events += self._process(prev)
                prev = None
            self.running = [s for s in self.running if not s.finished]
            dec = self._preempt_for_growth()
        B = len(dec)
        from_prev = None
        toks: List[int] = []
        pos: List[int] = []
        slot_parts: List[np.ndarray] = []
        dec_in = None
        if B:
            width = self.width
            bt = np.zeros((B, width), np.int32)
            cl = np.zeros(B, np.int32)
            sl = np.zeros(B, np.int32)
            ps = np.zeros(B, np.int32)
            prepare_decode_into(self.bm, [s.id for s in dec], width, B, bt, cl, sl, ps)
            prev_rows = {s.id: i for i, s in enumerate(prev.seqs)} if prev is not None else {}
            src = [(i, prev_rows[s.id]) for i, s in enumerate(dec) if s.id in prev_rows]
            if src:  # input tokens still on the device (the previous step's sampler output)
                from_prev = (_h2d([a for a, _ in src], torch.int64, dev), _h2d([b for _, b in src], torch.int64, dev))
            toks.extend(s.tokens[-1] if s.tokens else 0 for s in dec)
            pos.extend(ps.tolist())
            slot_parts.append(sl)
            dec_in = {"block_tables": _h2d(bt, torch.int32, dev), "ctx_lens": _h2d(cl, torch.int32, dev)}
            if self.prefix_sharing and B >= self.cascade_min_batch and self._cascade_pays(dec):
                per = ops.cascade_rows_per_tile(self.cfg.heads // self.cfg.kv_heads)
                tiles = np.zeros((cascade_table_size(B, per), 3), np.int32)
                self._cascade_plan(dec, tiles)
                dec_in["tiles"] = _h2d(tiles, torch.int32, dev)
            else:
                splits = min(max(1, min(16, -(-1024 // (B * self.cfg.kv_heads)))), max(1, self.width // 4))
                dec_in["splits"] = splits if self.decode_splits is None else int(self.decode_splits)
        cu, k_lens, tables, last_rows = [0], [], [], []
        for g, a, e in items:
            p = g.prompt_ids
            toks.extend(p[a:e])
            pos.extend(range(a, e))
            slot_parts.append(slots_range(self.bm, -g.id, a, e - a))
            cu.append(cu[-1] + e - a)
            k_lens.append(e)
            tables.append(list(self.bm.block_table(-g.id)))
            last_rows.append(B + cu[-1] - 1)
        wc = 2 * -(-max(k_lens) // 32)
        bt_c = np.zeros((len(items), wc), np.int32)
        for i, t in enumerate(tables):
            bt_c[i, :len(t)] = t[:wc]
        chunk_in = {"cu_q": _h2d(cu, torch.int32, dev), "block_tables": _h2d(bt_c, torch.int32, dev),
                    "k_lens": _h2d(k_lens, torch.int32, dev), "max_q": max(e - a for _, a, e in items),
                    "lens": ([e - a for _, a, e in items], k_lens)}
        copies = self.bm.take_copies()
        if copies:
            self.cache.copy_blocks(_h2d(copies, torch.int32, dev))
        rows = list(range(B)) + last_rows
        t_tok = _h2d(toks, torch.int32, dev)
        if from_prev is not None:
            t_tok.index_copy_(0, from_prev[0], prev.tok_dev.index_select(0, from_prev[1]).to(torch.int32))
        logits = self.model.forward_mixed(t_tok, _h2d(pos, torch.int32, dev),
                                          _h2d(np.concatenate(slot_parts), torch.int32, dev), self.cache, B, dec_in,
                                          chunk_in, _h2d(rows, torch.int64, dev))
        if prev is not None:  # host bookkeeping of the previous step while this forward runs
            with span("decode.process"):
                events += self._process(prev)
        self.stats["prefill_tokens"] += cu[-1]
        self.stats["prefill_chunks"] = self.stats.get("prefill_chunks", 0) + 1
        self.stats["mixed_steps"] = self.stats.get("mixed_steps", 0) + 1
        if B:
            self.stats["decode_tokens"] += B
            self.stats["steps"] += 1
        # prompts completed by this chunk: register their blocks in the prefix cache, fork their sequences
        done, pick = [], list(range(B))
        for i, (g, a, e) in enumerate(items):
            g.pf_pos = e
            if self.prefix_caching:  # register the blocks computed so far: prompts waiting on them can start
                self.bm.cache_prefix(-g.id, g.prompt_ids if e == len(g.prompt_ids) else g.prompt_ids[:e])
            if e == len(g.prompt_ids):
                done.append((g, B + i))
        children: List[Sequence] = []
        if done:
            ids = {g.id for g, _ in done}
            self.prefilling = [g for g in self.prefilling if g.id not in ids]
            for g, row in done:
                for s in g.seqs:
                    self.bm.fork(-g.id, s.id)
                    self._attach_rows(s)
                    children.append(s)
                    pick.append(row)
                self.bm.free_sequence(-g.id)
        seqs = dec + children
        if seqs:
            sel = logits if pick == list(range(logits.shape[0])) else logits.index_select(
                0, _h2d(pick, torch.int64, dev))
            self.inflight = self._launch_first(sel, seqs, [g for g, _ in done])
            self.running.extend(children)
            self._comp_cache = (None, None)
        return events

    def _block_chain(self, g: SequenceGroup) -> List[int]:
        """Chained hashes of the prompt's full blocks (block i's hash covers tokens [0, 16(i+1))), computed once
        per prompt: equal chains = a shared prefix, block for block."""
        ch = g._chain
        if ch is None:
            p, bs, h = g.prompt_ids, self.block_size, 0
            ch = []
            for i in range((len(p) - 1) // bs):
                h = hash((h, tuple(p[i * bs:(i + 1) * bs])))
                ch.append(h)
            g._chain = ch
        return ch

    def _tune_mixed(self) -> None:
        """Once, before the first mixed step: the GEMM backend per row-count bucket of the mixed steps'
        projections (decode rows + up to ``chunked_prefill`` chunk rows), timed like the decode buckets'.
        ``LWC_GEMM_BUCKETS``: ``swiglu`` (default) tunes the gate|up + SwiGLU projection only — the
        hand-written cores win it at every serving row count (profiles/serve_load.md, round 5: 4-7 %, and no
        separate silu_mul pass); ``1`` every projection (measured 28.0-28.9 vs 28.5-31.5 requests/s without in
        round 3: a bucket's choice is timed at its top row count, and for the few-tile o / down shapes
        hipBLASLt's stream-K is the safer pick across the row counts below it); ``0`` none."""
        self._mixed_tuned = True
        mode = os.environ.get("LWC_GEMM_BUCKETS", "swiglu")
        if not hasattr(self.model, "tune_gemms") or self.device.type != "cuda" or mode not in ("1", "swiglu"):
            return
        top = self.chunked_prefill + self.max_batch
        buckets = [m for m in (256, 512, 1024, 1536, 2048, 2560, 3072, 4096, 6144, 8192) if m < top] + [top]
        with span("tune_gemms"):
            for m in buckets:
                if mode == "1":
                    self.model.tune_gemms(m, bucket=True, lm_head=False)
                else:
                    self.model.tune_gemms(m, bucket=True, lm_head=False, only=("swiglu",))

    def _chunk_items(self, budget: int):
        """This step's prompt chunks: (group, a, e) = prompt tokens [a, e), at most ``budget`` tokens, prompts
        in admission order.  A prompt not started yet whose next uncached block another prompt in progress is
        about to compute (the voters of one score request share their messages head; every request shares
        the instructions) waits for it and then takes the shared blocks from the prefix cache — blocks are
        registered chunk by chunk, so it waits only until the shared part is computed, not the whole prompt."""
        bs = self.block_size
        items: List[Tuple[SequenceGroup, int, int]] = []
        deferred = False
        pending: set = set()  # chain hashes of blocks that prompts in progress have not computed yet
        if self.prefix_caching:
            for g in self.prefilling:
                if g.pf_pos >= 0:
                    ch = self._block_chain(g)
                    pending.update(ch[g.pf_pos // bs:])
        for g in self.prefilling:
            if budget <= 0:
                break
            p = g.prompt_ids
            if g.pf_pos < 0:
                if self.prefix_caching:
                    ch = self._block_chain(g)
                    k = int(self.bm.match_prefix(p)) // bs
                    if k < len(ch) and ch[k] in pending:
                        deferred = True
                        continue
                    g.pf_pos = int(self.bm.add_sequence_cached(-g.id, p))
                    self.stats["prefix_cache_tokens"] += g.pf_pos
                    pending.update(ch[g.pf_pos // bs:])
                else:
                    self.bm.add_sequence(-g.id, len(p))
                    g.pf_pos = 0
            n = min(budget, len(p) - g.pf_pos)
            items.append((g, g.pf_pos, g.pf_pos + n))
            budget -= n
        return items, budget, deferred

    def _drop_prefilling(self, g: SequenceGroup, reason: str) -> None:
        if g.pf_pos >= 0 and self.bm.has_sequence(-g.id):
            self.bm.free_sequence(-g.id)
        for s in g.seqs:
            s.finished, s.finish_reason = True, reason
        self.free_blocks_unreserved += g.reserved_blocks
        g.reserved_blocks = 0
        self.prefilling = [x for x in self.prefilling if x is not g]

    def _prefill_waves(self, groups: List[SequenceGroup]) -> List[List[SequenceGroup]]:
        """Split one admission batch so prompts that share a head INSIDE the batch (the voters of one
        score request: same messages, different key tails) compute it once: the first prompt of each
        shared head goes in wave 1, the prompts that would reuse more of it than the cache already holds
        go in wave 2 and take the head from the prefix cache wave 1 just filled."""
        if not self.prefix_caching or len(groups) < 2:
            return [groups] if groups else []
        bs = self.block_size
        leaders: Dict[tuple, np.ndarray] = {}
        first, second = [], []
        for g in groups:
            p = g.prompt_ids
            if len(p) <= bs:
                first.append(g)
                continue
            key = tuple(p[:bs])
            lead = leaders.get(key)
            if lead is None:
                leaders[key] = np.asarray(p, dtype=np.int64)
                first.append(g)
                continue
            a = np.asarray(p, dtype=np.int64)
            n = min(len(a), len(lead))
            diff = np.nonzero(a[:n] != lead[:n])[0]
            common = int(diff[0]) if diff.size else n
            shared = min(common, len(p) - 1) // bs * bs
            (second if shared > self.bm.match_prefix(p) else first).append(g)
        return [w for w in (first, second) if w]

    def _attach_rows(self, s: Sequence) -> None:
        p = s.params
        if p.uses_penalties:
            if self.counts is None:
                self.counts = torch.zeros(self.max_batch, self.cfg.vocab_size, dtype=torch.int16, device=self.device)
            s.count_row = self.free_count_rows.pop()
            self.counts[s.count_row].zero_()
        g = s.group
        if p.logit_bias and g.bias_row < 0:
            if self.bias is None:
                self.bias = torch.zeros(self.max_batch, self.cfg.vocab_size, dtype=torch.float32, device=self.device)
            g.bias_row = self.free_bias_rows.pop()
            row = torch.zeros(self.cfg.vocab_size, dtype=torch.float32)
            for k, v in p.logit_bias.items():
                row[int(k)] = float(v)
            self.bias[g.bias_row].copy_(row)
        if p.constraint is not None:
            s.constraint_state = p.constraint.start()

    # ------------------------------------------------------------------ decode
    def _bucket(self, B: int) -> _GraphBucket:
        Bb = next((b for b in BUCKETS if b >= B), None)
        if Bb is None:
            raise RuntimeError(f"batch {B} larger than the largest bucket")
        bk = self.buckets.get(Bb)
        if bk is None:
            # split-K so that a launch has >= ~1024 (batch, kv-head, split) workgroups
            splits = max(1, min(16, -(-1024 // (Bb * self.cfg.kv_heads))))
            splits = min(splits, max(1, self.width // 4))
            if self.decode_splits is not None:
                splits = int(self.decode_splits)
            max_tiles = 0
            if self.prefix_sharing and Bb >= self.cascade_min_batch:
                per = ops.cascade_rows_per_tile(self.cfg.heads // self.cfg.kv_heads)
                max_tiles = cascade_table_size(Bb, per)
            bk = _GraphBucket(Bb, self.width, splits, max_tiles, self.device)
            self.buckets[Bb] = bk
            if hasattr(self.model, "tune_gemms"):
                # per-shape GEMM backend (ops/gemm_plan.py), measured once per bucket, before any graph
                # of it is captured (graph and eager decode then run the same kernels)
                with span("tune_gemms"):
                    self.model.tune_gemms(Bb)
        return bk

    def _cascade_plan(self, seqs: List[Sequence], tiles: np.ndarray) -> None:
        """Super-tiles of the cascade decode kernel (see :func:`cascade_tiles`): runs of consecutive
        sequences forked from one prompt share the prompt's full blocks."""
        runs, i, B = [], 0, len(seqs)
        while i < B:
            g = seqs[i].group
            j = i
            while j < B and seqs[j].group is g:
                j += 1
            runs.append((i, j - i, len(g.prompt_ids) // self.block_size))
            i = j
        per = ops.cascade_rows_per_tile(self.cfg.heads // self.cfg.kv_heads)
        cascade_tiles(runs, per, tiles)

    def _static_inputs(self, seqs: List[Sequence], key, bk: _GraphBucket) -> dict:
        """Per-composition inputs (prefix tiles, sampler parameters), rebuilt only when the batch
        composition changes — in steady-state decoding only positions/slots/offsets move."""
        ck, cached = self._comp_cache
        if ck == key and cached is not None:
            return cached
        B = bk.B
        ps = [s.params for s in seqs]
        n = len(seqs)
        st = {"tiles": np.zeros((max(1, bk.max_tiles), 3), np.int32),
              "cascade": bool(bk.max_tiles) and self._cascade_pays(seqs)}
        if st["cascade"]:
            self._cascade_plan(seqs, st["tiles"])

        def col(vals, dt, fill=0):
            a = np.full(B, fill, dtype=dt)
            a[:n] = vals
            return a

        st["temperature"] = col([p.temperature for p in ps], np.float32, 1.0)
        st["top_p"] = col([p.top_p for p in ps], np.float32, 1.0)
        st["top_k"] = col([p.top_k for p in ps], np.int32)
        st["min_p"] = col([p.min_p for p in ps], np.float32)
        st["top_a"] = col([p.top_a for p in ps], np.float32)
        st["freq_pen"] = col([p.frequency_penalty for p in ps], np.float32)
        st["pres_pen"] = col([p.presence_penalty for p in ps], np.float32)
        st["rep_pen"] = col([p.repetition_penalty for p in ps], np.float32, 1.0)
        st["count_rows"] = col([s.count_row for s in seqs], np.int32, -1)
        st["bias_rows"] = col([s.group.bias_row for s in seqs], np.int32, -1)
        st["seeds"] = col([s.seed for s in seqs], np.int64)
        st["K"] = max((p.top_logprobs for p in ps), default=0)
        st["need_lp"] = any(p.logprobs for p in ps)
        st["any_pen"] = any(p.uses_penalties for p in ps)
        st["any_bias"] = any(s.group.bias_row >= 0 for s in seqs)
        self._comp_cache = (key, st)
        return st

    def _cascade_pays(self, seqs: List[Sequence]) -> bool:
        """Whether the cascade kernel beats plain split-K decode for this batch: at least half of its rows
        belong to runs of >= 2 sequences forked from one prompt (candidates of one request).  Batches of
        unrelated sequences (the voters of score requests are separate n = 1 requests) would run the cascade
        kernel as plain decode with one wave walking 16/G whole contexts — few, long-serial workgroups."""
        shared, i, B = 0, 0, len(seqs)
        while i < B:
            g = seqs[i].group
            j = i
            while j < B and seqs[j].group is g:
                j += 1
            if j - i >= 2 and len(g.prompt_ids) >= self.block_size:
                shared += j - i
            i = j
        return 2 * shared >= B

    def _ensure_graph(self, bk: _GraphBucket, cascade: Optional[bool] = None) -> None:
        d = bk.d
        cascade = bool(bk.max_tiles) if cascade is None else cascade

        def fwd():
            return self.model.decode(d["tokens"], d["positions"], d["slots"], d["block_tables"], d["ctx_lens"],
                                     self.cache, num_splits=bk.splits,
                                     cascade_tiles=d["tiles"] if cascade else None)

        if not self.use_graphs:
            bk.logits = fwd()
            return
        g = bk.graphs.get(cascade)
        if g is None and not bk.graphs and bk.B not in self.step_ab:
            self._step_ab(bk, fwd)
        if g is None:
            dev = self.device
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                fwd()  # warm-up (hipBLASLt heuristics, allocator) outside capture
            torch.cuda.current_stream(dev).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            # thread_local: another thread's device work during this capture (the K10b tally batcher's
            # launches, allocations and read-backs on its own stream, score/tally_batch.py) neither
            # invalidates the capture nor fails itself; only this thread's calls are checked
            with torch.cuda.graph(g, pool=bk.pool, capture_error_mode="thread_local"):
                bk.graph_logits[cascade] = fwd()  # (the bucket's two graphs never run at once)
            bk.pool = g.pool()
            bk.graphs[cascade] = g
            bk.graph = g
        bk.logits = bk.graph_logits[cascade]
        g.replay()

    def _step_ab(self, bk: _GraphBucket, fwd) -> None:
        """In-step A/B of the model's plans for this bucket: every candidate is captured into a graph of its own
        and replayed on this step's real inputs (a decode replay rewrites the same KV slots with the same
        values, nothing else); the median of 5 replays ranks it.  Round 1 ranks whole plans (``step_plans``: the
        isolated planner's choice, all-library, all-hand-written); then one coordinate-descent pass over
        single-decision moves from the best (``step_moves``: one projection's backend, one norm point folded or
        not, a consumer's schedule, a producer's mode), each kept when it beats the incumbent by more than
        0.2 %.  Isolated per-GEMM timings do not see the step's clock and cache state (they flipped choices
        that lost 0.5 % in the bench); this measures the thing that runs.  ``LWC_STEP_AB=0`` keeps the
        planner's choice, ``LWC_STEP_AB=plans`` skips the moves, ``LWC_STEP_PLAN=<name>`` runs that whole plan
        (profiling).  Decided once per model and batch; results in ``self.step_ab[B]`` and on stderr.
        Only for buckets of at least ``LWC_STEP_AB_MIN`` rows (default 1024): below, the projections are few-tile
        or weight-streaming shapes the planner's isolated timings rank the same way, and a serving engine
        meets many small buckets — each A/B captures ~20 graphs (measured: ~10 s of a 256-request load test)."""
        self.step_ab[bk.B] = {}
        mode = os.environ.get("LWC_STEP_AB", "1")
        if mode == "0" or not hasattr(self.model, "step_plans"):
            return
        if bk.B < int(os.environ.get("LWC_STEP_AB_MIN", "1024")) and not os.environ.get("LWC_STEP_PLAN"):
            return
        if getattr(self.model, "tp_size", 1) > 1 or getattr(self.model, "ep_size", 1) > 1:
            # a tensor- / expert-parallel step holds collectives: every rank would have to capture and replay
            # the same candidates in the same order, and each rank's candidates come from its own timings
            return
        # every engine on the model then runs the same kernels (engines compared against each other)
        done = self.model.__dict__.setdefault("step_ab_done", {})
        if bk.B in done:
            self.step_ab[bk.B] = done[bk.B]
            return
        plans = self.model.step_plans(bk.B)
        if len(plans) < 2:
            return
        dev = self.device
        s = torch.cuda.Stream(device=dev)

        def capture(plan):
            self.model.apply_step_plan(bk.B, plan)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                fwd()  # warm-up outside capture (first launches of new kernels set their attributes)
            torch.cuda.current_stream(dev).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                out = fwd()
            g.replay()
            return g, out

        def replay_ms(g) -> float:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1)

        def race(graphs: dict, rounds: int = 4, raw: bool = False) -> dict:
            # interleaved replays (ABAB...): the clock's drift hits every candidate alike; median per candidate
            ts = {k: [] for k in graphs}
            for _ in range(rounds):
                for k, (g, _) in graphs.items():
                    ts[k].append(replay_ms(g))
            return ts if raw else {k: sorted(v)[len(v) // 2] for k, v in ts.items()}

        def try_capture(name, plan):
            # a candidate that fails to build or capture (a kernel refusing its shape, say) drops out of the
            # race instead of failing the engine; the planner's own plan is what ran before the A/B existed
            try:
                return capture(plan)
            except RuntimeError as e:
                print(f"# step A/B at batch {bk.B}: candidate {name} dropped ({e})", file=sys.stderr, flush=True)
                return None

        graphs = {name: g for name, g in ((n, try_capture(n, p)) for n, p in plans.items()) if g is not None}
        if not graphs:
            self.model.apply_step_plan(bk.B, plans["planner"])
            return
        times = race(graphs, 5)
        best = min(times, key=times.get)
        cur, t_cur = plans[best], times[best]
        inc = graphs.pop(best)
        del graphs
        kept = []
        if mode != "plans" and hasattr(self.model, "step_moves"):
            # coordinate descent: each move raced against the incumbent (both graphs alive, 6 paired rounds);
            # kept when the median move / incumbent ratio says > 0.25 % faster, and it becomes the incumbent
            for label, delta in self.model.step_moves(bk.B, cur):
                cand = self.model.with_move(cur, delta)
                gm = try_capture(label, cand)
                if gm is None:
                    continue
                # paired: the median of the per-round move / incumbent ratios (back-to-back replays share the
                # clock state; separate medians let a no-op move "win" by 0.3 %)
                r = race({"inc": inc, "mv": gm}, 6, raw=True)
                ratios = sorted(a / b for a, b in zip(r["mv"], r["inc"]))
                ratio = 0.5 * (ratios[len(ratios) // 2 - 1] + ratios[len(ratios) // 2])
                times[label] = ratio * t_cur  # on the incumbent's scale
                if ratio < 0.9975:
                    cur, inc, t_cur = cand, gm, times[label]
                    kept.append(label)
                else:
                    del gm
        del inc
        forced = os.environ.get("LWC_STEP_PLAN")
        if forced in plans:
            cur, kept = plans[forced], [f"forced {forced}"]
        self.model.apply_step_plan(bk.B, cur)
        torch.cuda.empty_cache()
        self.step_ab[bk.B] = done[bk.B] = dict({k: round(v, 3) for k, v in times.items()}, choice=best,
                                                moves=kept, final=round(t_cur, 3))
        plan = self.model.plan_summary(bk.B) if hasattr(self.model, "plan_summary") else {}
        print(f"# step A/B at batch {bk.B}: " + " ".join(f"{k}={v:.2f}ms" for k, v in times.items())
              + f" -> {best} + {kept} ({t_cur:.2f} ms) {plan}", file=sys.stderr, flush=True)

    def _launch(self, seqs: List[Sequence], sample: bool = True) -> _Step:
        """Stage inputs, replay the decode graph and launch the sampler for `seqs`; results are
        copied to pinned host memory asynchronously (processed later by :meth:`_process`).
        ``sample=False`` stops after the forward: :meth:`_launch_sample` launches the sampler later
        (constrained batches: their grammar masks need the previous step's tokens on the host, which
        are processed while this forward runs)."""
        B = len(seqs)
        bk = self._bucket(B)
        key = (bk.B, tuple(s.id for s in seqs))
        parity = self._step_no & 1
        self._step_no += 1
        h = bk.h[parity]
        prepare_decode_into(self.bm, [s.id for s in seqs], bk.width, bk.B, h["block_tables"], h["ctx_lens"],
                            h["slots"], h["positions"])
        st = self._static_inputs(seqs, key, bk)
        if bk.host_static_key[parity] != key:
            for name in ("tiles", "seeds") + _F32_PARAMS + _I32_PARAMS:
                h[name][...] = st[name]
            bk.host_static_key[parity] = key
        prev = self.inflight
        prev_rows = {}
        if prev is not None and prev.key != key:
            prev_rows = {s.id: i for i, s in enumerate(prev.seqs)}
        offs = h["offsets"]
        tok_h = h["tokens"]
        from_prev_dst, from_prev_src = [], []
        same = prev is not None and prev.key == key
        for i, s in enumerate(seqs):
            offs[i] = s.n_launched
            if not same:
                if len(s.tokens) == s.n_launched:
                    tok_h[i] = s.tokens[-1]
                else:  # last token still in flight: take it from the previous step's device output
                    from_prev_dst.append(i)
                    from_prev_src.append(prev_rows[s.id])
            s.n_launched += 1
        dev = self.device
        copies = self.bm.take_copies()
        bk.dev.copy_(bk.host[parity], non_blocking=True)
        d = bk.d
        if same:
            d["tokens"][:B].copy_(prev.tok_dev[:B])
        elif from_prev_dst:
            dst = torch.tensor(from_prev_dst, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
            src = torch.tensor(from_prev_src, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
            d["tokens"].index_copy_(0, dst, prev.tok_dev.index_select(0, src))
        if copies:
            self.cache.copy_blocks(_h2d(copies, torch.int32, dev))
        self._ensure_graph(bk, st["cascade"])
        self._comm_arm()  # TP: error word of this step's all-reduces -> pinned host memory, read one step later
        step = _Step(seqs, key, bk, parity, st["K"], None, None, None)
        step.static = st
        self.stats["decode_tokens"] += B
        self.stats["steps"] += 1
        if sample:
            self._launch_sample(step)
        return step

    def _launch_sample(self, step: _Step) -> None:
        """Launch the sampler of a launched forward (grammar masks from the sequences' current
        constraint states) and the asynchronous copy of its outputs to pinned host memory."""
        seqs, bk, parity, st = step.seqs, step.bk, step.parity, step.static
        B, K, d = len(seqs), step.K, bk.d
        mask = mask_rows = None
        cons = [i for i, s in enumerate(seqs) if s.constraint_state is not None]
        if cons:
            mask, mask_rows = self._constraint_masks(seqs, cons)
        outs, out_dev, out_host = bk.outputs(parity, K)
        ops.sample(bk.logits[:B], temperature=d["temperature"], top_p=d["top_p"], top_k=d["top_k"],
                   min_p=d["min_p"], top_a=d["top_a"], seeds=d["seeds"], offsets=d["offsets"], num_logprobs=K,
                   freq_pen=d["freq_pen"] if st["any_pen"] else None,
                   pres_pen=d["pres_pen"] if st["any_pen"] else None,
                   rep_pen=d["rep_pen"] if st["any_pen"] else None,
                   counts=self.counts if st["any_pen"] else None,
                   count_rows=d["count_rows"] if st["any_pen"] else None,
                   bias=self.bias if st["any_bias"] else None,
                   bias_rows=d["bias_rows"] if st["any_bias"] else None,
                   mask=mask, mask_rows=mask_rows, mask_logprobs=self.constrained_logprobs,
                   need_logprob=st["need_lp"], out_token=outs[0], out_logprob=outs[1], out_topk_ids=outs[2], out_topk_lp=outs[3])
        out_host.copy_(out_dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        step.tok_dev, step.out_host, step.event = outs[0], out_host, ev

    def _constraint_masks(self, seqs: List[Sequence], cons: List[int]):
        """(mask table [rows, V/32] int32 on the device, per-sequence row [B] int32).

        Each constraint maps its FSM state to a cached full-vocabulary token mask + content digest
        (:meth:`TokenConstraint.mask_entry`).  Masks are keyed by that digest: every distinct mask is
        uploaded ONCE into a device-resident table (the voters of a score request, each with its own
        shuffled key enum, still share most states: '{', the property name, quotes, ...), and a step
        uploads only the B row indices."""
        if self._mask_rows_of is None:
            self._mask_rows_of = {}
            self._mask_table = torch.zeros(64, self.cfg.vocab_size // 32, dtype=torch.int32, device=self.device)
        rows = np.full(len(seqs), -1, dtype=np.int32)
        new: List[Tuple[int, np.ndarray]] = []
        for i in cons:
            s = seqs[i]
            ent = s.params.constraint.mask_entry(s.constraint_state)
            key = ent.key
            r = self._mask_rows_of.get(key)
            if r is None:
                if len(self._mask_rows_of) >= self._mask_limit:  # bounded: start the table over
                    self._mask_rows_of.clear()
                    return self._constraint_masks(seqs, cons)
                r = len(self._mask_rows_of)
                self._mask_rows_of[key] = r
                new.append((r, ent.words()))
            rows[i] = r
        if new:
            need = max(r for r, _ in new) + 1
            if need > self._mask_table.shape[0]:
                grown = torch.zeros(max(need, 2 * self._mask_table.shape[0]), self._mask_table.shape[1],
                                    dtype=torch.int32, device=self.device)
                grown[:self._mask_table.shape[0]] = self._mask_table
                self._mask_table = grown
            # pinned + non_blocking: a pageable upload synchronises the stream, i.e. would wait for the
            # decode forward already queued ahead of the sampler
            self._mask_table.index_copy_(0, _h2d([r for r, _ in new], torch.int64, self.device),
                                         _h2d(np.stack([m for _, m in new]).view(np.int32), torch.int32, self.device))
        return self._mask_table, _h2d(rows, torch.int32, self.device)

    def _process(self, st: _Step) -> List[TokenEvent]:
        st.event.synchronize()
        self._comm_poll()  # a TP peer that never arrived: CommFailure fails the in-flight groups (EngineService)
        if st.first is not None:  # first tokens after a prefill (:meth:`_launch_first`)
            host, groups = st.first
            lists = [h.tolist() for h in host]
            events = self._advance(st.seqs, lists[0], lists[1], lists[2] if st.K else None,
                                   lists[3] if st.K else None)
            for g in groups:
                g.timer.token()
            return events
        B, K = len(st.seqs), st.K
        Kb = max(K, 1)
        Bp = st.bk.B
        a = st.out_host.numpy()
        tok_h = a[:B].tolist()
        lp_h = a[Bp:Bp + B].view(np.float32).tolist()
        if K:
            ids_h = a[2 * Bp:2 * Bp + Bp * Kb].reshape(Bp, Kb)[:B, :K].tolist()
            lps_h = a[2 * Bp + Bp * Kb:2 * Bp + 2 * Bp * Kb].view(np.float32).reshape(Bp, Kb)[:B, :K].tolist()
        else:
            ids_h = lps_h = None
        return self._advance(st.seqs, tok_h, lp_h, ids_h, lps_h)

    def _drain(self) -> List[TokenEvent]:
        st, self.inflight = self.inflight, None
        if st is None:
            return []
        events = self._process(st)
        self.running = [s for s in self.running if not s.finished]
        return events

    def _decode(self) -> List[TokenEvent]:
        events: List[TokenEvent] = []
        # grammar masks depend on the previous token: a constrained batch launches its forward first
        # (its input tokens come from the previous step's device output), processes the previous step on
        # the host while that forward runs, and only then launches the sampler with the new masks
        constrained = any(s.constraint_state is not None for s in self.running)
        seqs = [s for s in self.running if not s.finished and s.n_launched < s.params.max_tokens]
        if not seqs:
            return events + self._drain()
        if self.bm.append_cost_total([s.id for s in seqs]) > self.bm.num_free:
            events += self._drain()  # nothing in flight: sequences can leave the batch
            seqs = self._preempt_for_growth()
            if not seqs:
                return events
            constrained = any(s.constraint_state is not None for s in self.running)
        with span("decode.launch"):
            cur = self._launch(seqs, sample=not constrained)
        prev, self.inflight = self.inflight, cur
        if prev is not None:
            with span("decode.process"):
                events += self._process(prev)
        if constrained:
            self._launch_sample(cur)
        self.running = [s for s in self.running if not s.finished]
        return events

    # ------------------------------------------------------------------ preemption (swap)
    def _preempt_for_growth(self) -> List[Sequence]:
        """Swap out the youngest running groups until one decode step of the rest fits the free pool;
        returns the sequences left to decode.  Called with no step in flight."""
        while True:
            seqs = [s for s in self.running if not s.finished and s.n_launched < s.params.max_tokens]
            if not seqs or self.bm.append_cost_total([s.id for s in seqs]) <= self.bm.num_free:
                return seqs
            groups = sorted({s.group.id: s.group for s in self.running if not s.finished}.values(),
                            key=lambda g: g.id)
            if len(groups) <= 1:
                raise RuntimeError("KV cache exhausted by a single request (raise num_blocks or lower max_tokens)")
            self._swap_out(groups[-1])

    def _swap_out(self, g: SequenceGroup) -> None:
        live = [s for s in g.seqs if not s.finished and self.bm.has_sequence(s.id)]
        blocks, tables, lens = self.bm.swap_out([s.id for s in live])
        dev = self.device
        if blocks:
            kv = self.cache.pool.index_select(2, torch.tensor(blocks, dtype=torch.int64, device=dev))
            host = torch.empty(kv.shape, dtype=kv.dtype, pin_memory=dev.type == "cuda")
            host.copy_(kv, non_blocking=True)  # stream-ordered before any later write to the freed blocks
        else:
            host = torch.empty(0)
        ev = None
        if dev.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        self.swapped.append(_SwapRecord(g, live, host, [list(t) for t in tables], list(lens), ev))
        ids = {s.id for s in live}
        self.running = [s for s in self.running if s.id not in ids]
        self.free_blocks_unreserved += g.reserved_blocks
        g.reserved_blocks = 0
        self._comp_cache = (None, None)
        self.stats["preemptions"] += 1
        self.stats["swapped_blocks"] += len(blocks)

    def _swap_in(self) -> None:
        """Resume preempted groups, oldest preemption first, while the pool holds them (plus one growth
        block per sequence and the watermark)."""
        while self.swapped:
            rec = self.swapped[0]
            n = rec.host.shape[2] if rec.host.dim() == 4 else 0
            need = self._group_reservation(rec.group)
            if (n + len(rec.seqs) + self.kv_watermark > self.bm.num_free
                    or (need > self.free_blocks_unreserved and (self.running or self.inflight is not None))):
                return
            self.swapped.popleft()
            phys = self.bm.swap_in([s.id for s in rec.seqs], n, rec.tables, rec.lens)
            if n:
                dev = self.device
                kv = rec.host.to(dev, non_blocking=True)
                self.cache.pool.index_copy_(2, torch.tensor(phys, dtype=torch.int64, device=dev), kv)
            rec.group.reserved_blocks = need
            self.free_blocks_unreserved -= need
            self.running.extend(s for s in rec.seqs if not s.finished)
            self._comp_cache = (None, None)

    # ------------------------------------------------------------------ sampling + bookkeeping
    def _sample_and_advance(self, logits: torch.Tensor, seqs: List[Sequence]) -> List[TokenEvent]:
        """Synchronous sampling (first token after prefill)."""
        tok, lp, tk_ids, tk_lp, K = self._sample_first(logits, seqs)
        self._comm_arm()
        host = [t.cpu().tolist() for t in ((tok, lp, tk_ids, tk_lp) if K else (tok, lp))]
        self._comm_poll()  # the .cpu() reads synchronised the stream: the armed error word is on the host
        return self._advance(seqs, host[0], host[1], host[2] if K else None, host[3] if K else None)

    def _comm_arm(self) -> None:
        """TP / EP models: queue the readback of the collectives' error word behind the work launched so far.
        Every step whose tokens reach the host is armed (decode replays, mixed chunked-prefill steps,
        prefills): :meth:`_process` polls it before advancing that step's tokens, so tokens sampled from a
        forward whose all-reduce was poisoned by a missing peer are never delivered."""
        arm = getattr(self.model, "comm_arm", None)
        if arm is not None:
            arm()

    def _comm_poll(self) -> None:
        poll = getattr(self.model, "comm_poll", None)
        if poll is not None:
            poll()

    def _launch_first(self, logits: torch.Tensor, seqs: List[Sequence], groups: List[SequenceGroup]) -> _Step:
        """Asynchronous first-token sampling after a prefill: the sampler and the copy of its outputs
        to pinned host memory are queued and the result becomes the in-flight step, processed by the
        next decode step after it has launched its own forward — the GPU goes from the prefill
        straight into the next decode step instead of idling while the host forks and advances."""
        tok, lp, tk_ids, tk_lp, K = self._sample_first(logits, seqs)
        host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in ((tok, lp, tk_ids, tk_lp) if K else
                                                                               (tok, lp))]
        for h, t in zip(host, (tok, lp, tk_ids, tk_lp)):
            h.copy_(t, non_blocking=True)
        self._comm_arm()  # the prefill / mixed forward's collectives: checked by _process before these tokens
        ev = torch.cuda.Event()
        ev.record()
        st = _Step(seqs, None, None, 0, K, tok, None, ev)
        st.first = (host, groups)
        return st

    def _sample_first(self, logits: torch.Tensor, seqs: List[Sequence]):
        """Launch the sampler over prefill last-token logits (no host sync); advances n_launched."""
        B = len(seqs)
        dev = self.device
        ps = [s.params for s in seqs]
        f32 = lambda xs: torch.tensor(xs, dtype=torch.float32).pin_memory().to(dev, non_blocking=True)
        i32 = lambda xs: torch.tensor(xs, dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
        i64 = lambda xs: torch.tensor(xs, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
        K = max((p.top_logprobs for p in ps), default=0)
        any_pen = any(p.uses_penalties for p in ps)
        any_bias = any(s.group.bias_row >= 0 for s in seqs)
        cons = [i for i, s in enumerate(seqs) if s.constraint_state is not None]
        mask = mask_rows = None
        if cons:
            mask, mask_rows = self._constraint_masks(seqs, cons)
        tok, lp, tk_ids, tk_lp = ops.sample(
            logits,
            temperature=f32([p.temperature for p in ps]),
            top_p=f32([p.top_p for p in ps]),
            top_k=i32([p.top_k for p in ps]),
            min_p=f32([p.min_p for p in ps]),
            top_a=f32([p.top_a for p in ps]),
            seeds=i64([s.seed for s in seqs]),
            offsets=i64([s.n_launched for s in seqs]),
            num_logprobs=K,
            freq_pen=f32([p.frequency_penalty for p in ps]) if any_pen else None,
            pres_pen=f32([p.presence_penalty for p in ps]) if any_pen else None,
            rep_pen=f32([p.repetition_penalty for p in ps]) if any_pen else None,
            counts=self.counts if any_pen else None,
            count_rows=i32([s.count_row for s in seqs]) if any_pen else None,
            bias=self.bias if any_bias else None,
            bias_rows=i32([s.group.bias_row for s in seqs]) if any_bias else None,
            mask=mask, mask_rows=mask_rows, mask_logprobs=self.constrained_logprobs,
            need_logprob=any(p.logprobs for p in ps),
        )
        for s in seqs:
            s.n_launched += 1
        return tok, lp, tk_ids, tk_lp, K

    def _advance(self, seqs: List[Sequence], tok_h, lp_h, ids_h, lps_h) -> List[TokenEvent]:
        """Host bookkeeping of one sampled token per sequence: append, grammar advance, stop / length
        checks, and — only where someone consumes it — incremental detokenisation and a TokenEvent
        (a callback, or ``collect_events``).  The common batch path is an append and two compares."""
        events = []
        eos = self.tokenizer.eos_token_id
        collect = self.collect_events
        for i, s in enumerate(seqs):
            if s.finished:  # finished (or aborted) while this step was in flight: discard the row
                continue
            t = int(tok_h[i])
            p = s.params
            s.tokens.append(t)
            if s.constraint_state is not None:
                s.constraint_state = p.constraint.advance(s.constraint_state, t)
            cb = s.group.callback
            reason = None
            text = ""
            if t == eos and not p.ignore_eos:
                reason = "stop"
            elif p.stop_token_ids and t in p.stop_token_ids:
                reason = "stop"
            elif cb is not None or p.stop:
                if s._text is None:
                    s._text = ""
                text = s.detok.push(t)
                s._text += text
                if p.stop:
                    for st in p.stop:
                        k = s._text.find(st)
                        if k >= 0:
                            cut = len(s._text) - k
                            text = text[: max(0, len(text) - cut)]
                            s._text = s._text[:k]
                            reason = "stop"
                            break
            if reason is None and s.constraint_state is not None and p.constraint.is_done(s.constraint_state):
                reason = "stop"
            if reason is None and len(s.tokens) >= p.max_tokens:
                reason = "length"
            if cb is None and not collect:
                if reason is not None:
                    self._finish(s, reason)
                continue
            k = p.top_logprobs
            top = [(a, v) for a, v in zip(ids_h[i][:k], lps_h[i][:k]) if a >= 0] if k else []
            lp = float(lp_h[i])
            if self.faults.bad_logprobs:
                lp, top = float("nan"), [(a, float("nan")) for a, _ in top]
            ev = TokenEvent(s, t, text, lp, top)
            if reason is not None:
                self._finish(s, reason)
                ev.finished, ev.finish_reason = True, reason
            if collect:
                events.append(ev)
            if cb is not None:
                cb(ev)
        return events

    def _finish(self, s: Sequence, reason: str) -> None:
        s.finished = True
        s.finish_reason = reason
        self.bm.free_sequence(s.id)
        if s.count_row >= 0:
            self.free_count_rows.append(s.count_row)
            s.count_row = -1
        g = s.group
        if g.finished:
            g.timer.tokens = max(len(x.tokens) for x in g.seqs)
            g.timer.t_last = time.perf_counter()
            g.timer.finished()
            self.free_blocks_unreserved += g.reserved_blocks
            g.reserved_blocks = 0
            if g.bias_row >= 0:
                self.free_bias_rows.append(g.bias_row)
                g.bias_row = -1

    # ------------------------------------------------------------------ deadlines
    def expire(self, now: Optional[float] = None) -> List[SequenceGroup]:
        """Drop every group whose request deadline has passed — waiting, prefilling, preempted or
        generating (aborted between steps) — and return them; the caller tells their clients."""
        if not self._deadlines:
            return []
        now = time.monotonic() if now is None else now

        def late(g):
            return g.deadline is not None and now >= g.deadline and not g.finished

        out = []
        with self.lock:
            for g in [g for g in self.waiting if late(g)]:
                self.waiting.remove(g)
                for s in g.seqs:
                    s.finished, s.finish_reason = True, "deadline"
                out.append(g)
        seen = set()
        for g in [g for g in self.prefilling if late(g)] + [r.group for r in self.swapped if late(r.group)] + \
                [s.group for s in self.running if late(s.group)]:
            if g.id not in seen:
                seen.add(g.id)
                self.abort(g)
                for s in g.seqs:
                    s.finish_reason = "deadline"
                out.append(g)
        return out

    # ------------------------------------------------------------------ cancellation / failure
    def abort(self, g: SequenceGroup) -> None:
        """Drop a group (client went away): frees its blocks and reservation, no more events."""
        with self.lock:
            if g in self.waiting:
                self.waiting.remove(g)
                for s in g.seqs:
                    s.finished, s.finish_reason = True, "abort"
                return
        if any(x is g for x in self.prefilling):
            self._drop_prefilling(g, "abort")
            return
        rec = next((r for r in self.swapped if r.group is g), None)
        if rec is not None:  # preempted: its blocks are already free, only the host copy goes
            self.swapped.remove(rec)
            for s in g.seqs:
                if not s.finished:
                    s.finished, s.finish_reason = True, "abort"
                    if s.count_row >= 0:
                        self.free_count_rows.append(s.count_row)
                        s.count_row = -1
            if g.bias_row >= 0:
                self.free_bias_rows.append(g.bias_row)
                g.bias_row = -1
            return
        for s in g.seqs:
            if not s.finished:
                self._finish(s, "abort")
        self.running = [s for s in self.running if not s.finished]

    def fail_all(self, msg: str) -> List[SequenceGroup]:
        """After an engine exception: finish every in-flight group and return them."""
        groups = {}
        with self.lock:
            for g in self.waiting:
                groups[g.id] = g
            self.waiting.clear()
        for g in list(self.prefilling):
            groups[g.id] = g
            try:
                self._drop_prefilling(g, "error")
            except Exception:  # pragma: no cover - best effort cleanup
                pass
        self.prefilling = []
        for rec in list(self.swapped):
            groups[rec.group.id] = rec.group
            for s in rec.seqs:
                s.finished, s.finish_reason = True, "error"
        self.swapped.clear()
        for s in self.running:
            groups[s.group.id] = s.group
        for g in groups.values():
            for s in g.seqs:
                if not s.finished:
                    try:
                        self._finish(s, "error")
                    except Exception:  # pragma: no cover - best effort cleanup
                        s.finished = True
        self.running = []
        self.inflight = None
        self._comp_cache = (None, None)
        return list(groups.values())
