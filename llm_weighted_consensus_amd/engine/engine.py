"""Continuous-batching generation engine for one MI355X (one process per GPU).

This is the in-process replacement of the reference's upstream-provider round trip
(src/chat/completions/client.rs:193-434): a request becomes a *sequence group* of n sequences that
share their prompt's KV blocks (prefill once, fork n times — the multichat/voter fan-out of
src/score/completions/client.rs:343-356 mapped onto one GPU), and every `step()` advances all running
sequences by one token with a single batched decode launch.

Host runtime pieces are native C++ (`_runtime.BlockManager`: ref-counted paged-KV blocks with
copy-on-write fork, `prepare_decode`: per-step batch tables).  The decode forward is captured once per
batch bucket into a hipGraph (torch.cuda.CUDAGraph on ROCm) so a step is one graph replay plus the
fused sampler launch.

Admission control reserves worst-case KV for (prompt + n * max_tokens), so a running sequence can
never run out of blocks and no preemption path is needed; 288 GB of HBM3E makes this cheap.
"""
from __future__ import annotations

import itertools
import random
import threading
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Deque, Dict, List, Optional, Sequence as Seq, Tuple

import numpy as np
import torch

from .. import ops
from .._runtime import BlockManager, prepare_decode, slots_range
from ..models.llama import KVCache
from .sampling import SamplingParams
from .tokenizer import IncrementalDecoder

BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128, 256, 384, 512, 768, 1024)


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
        self.tokens: List[int] = []
        self.text = ""
        self.finished = False
        self.finish_reason: Optional[str] = None
        self.count_row = -1
        self.constraint_state = None
        self.detok = IncrementalDecoder(group.engine.tokenizer)

    @property
    def params(self) -> SamplingParams:
        return self.group.params


class SequenceGroup:
    _ids = itertools.count(1)

    def __init__(self, engine: "LLMEngine", prompt_ids: List[int], params: SamplingParams, n: int,
                 callback: Optional[Callable[[TokenEvent], None]]):
        self.id = next(SequenceGroup._ids)
        self.engine = engine
        self.prompt_ids = list(prompt_ids)
        self.params = params
        self.n = n
        self.callback = callback
        base = params.seed if params.seed is not None else random.getrandbits(63)
        self.seqs = [Sequence(self, i, (base * 1000003 + i) & ((1 << 63) - 1)) for i in range(n)]
        self.bias_row = -1
        self.reserved_blocks = 0

    @property
    def finished(self) -> bool:
        return all(s.finished for s in self.seqs)


class _GraphBucket:
    def __init__(self, B: int, width: int, splits: int, max_tiles: int):
        self.B, self.width, self.splits, self.max_tiles = B, width, splits, max_tiles
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.tokens = self.positions = self.slots = self.block_tables = self.ctx_lens = None
        self.tiles = self.start_blk = None
        self.logits: Optional[torch.Tensor] = None


class LLMEngine:
    def __init__(self, model, tokenizer, *, block_size: int = 16, num_blocks: Optional[int] = None,
                 kv_memory_fraction: float = 0.85, max_batch: int = 512, max_model_len: int = 4096,
                 use_graphs: bool = True, prefill_token_budget: int = 16384, prefix_sharing: bool = True):
        self.model = model
        self.cfg = model.cfg
        self.tokenizer = tokenizer
        self.device = model.device
        self.block_size = block_size
        self.max_batch = max_batch
        self.max_model_len = max_model_len
        self.prefill_token_budget = prefill_token_budget
        self.width = (max_model_len + block_size - 1) // block_size
        if num_blocks is None:
            free, _total = torch.cuda.mem_get_info(self.device)
            per = KVCache.bytes_per_block(self.cfg, block_size)
            num_blocks = max(64, int(free * kv_memory_fraction) // per)
        self.cache = KVCache(self.cfg, num_blocks, block_size, self.device)
        self.bm = BlockManager(num_blocks, block_size)
        self.free_blocks_unreserved = num_blocks
        self.use_graphs = use_graphs
        self.prefix_sharing = prefix_sharing
        self.buckets: Dict[int, _GraphBucket] = {}
        self.waiting: Deque[SequenceGroup] = deque()
        self.running: List[Sequence] = []
        self.lock = threading.Lock()
        V = self.cfg.vocab_size
        self.counts: Optional[torch.Tensor] = None  # [max_batch, V] int16, lazily
        self.free_count_rows = list(range(max_batch))
        self.bias: Optional[torch.Tensor] = None    # [max_batch, V] f32, lazily
        self.free_bias_rows = list(range(max_batch))
        self.stats = {"prefill_tokens": 0, "decode_tokens": 0, "steps": 0}

    # ------------------------------------------------------------------ API
    def add_request(self, prompt_ids: Seq[int], params: SamplingParams, n: int = 1,
                    callback: Optional[Callable[[TokenEvent], None]] = None) -> SequenceGroup:
        params.validate(self.cfg.vocab_size)
        if len(prompt_ids) == 0:
            raise ValueError("empty prompt")
        if len(prompt_ids) + params.max_tokens > self.max_model_len:
            raise ValueError(f"prompt ({len(prompt_ids)}) + max_tokens ({params.max_tokens}) exceeds "
                             f"max_model_len ({self.max_model_len})")
        g = SequenceGroup(self, list(prompt_ids), params, n, callback)
        with self.lock:
            self.waiting.append(g)
        return g

    def has_work(self) -> bool:
        return bool(self.waiting) or bool(self.running)

    def step(self) -> List[TokenEvent]:
        """Run one engine iteration: admit+prefill waiting groups if any fit, else one decode step."""
        with self.lock:
            admitted = self._admit()
        if admitted:
            return self._prefill(admitted)
        if self.running:
            return self._decode()
        return []

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
        per_child = (len(g.prompt_ids) + g.params.max_tokens + bs - 1) // bs - len(g.prompt_ids) // bs
        return prompt_blocks + g.n * (per_child + 1)

    def _admit(self) -> List[SequenceGroup]:
        out, tokens = [], 0
        while self.waiting:
            g = self.waiting[0]
            need = self._group_reservation(g)
            if len(self.running) + sum(x.n for x in out) + g.n > self.max_batch:
                break
            if need > self.free_blocks_unreserved:
                if not self.running and not out:
                    self.waiting.popleft()
                    raise RuntimeError("request needs more KV blocks than the cache holds")
                break
            if out and tokens + len(g.prompt_ids) > self.prefill_token_budget:
                break
            self.waiting.popleft()
            g.reserved_blocks = need
            self.free_blocks_unreserved -= need
            tokens += len(g.prompt_ids)
            out.append(g)
        return out

    # ------------------------------------------------------------------ prefill
    def _prefill(self, groups: List[SequenceGroup]) -> List[TokenEvent]:
        dev = self.device
        toks, pos, slots, cu, last = [], [], [], [0], []
        for g in groups:
            L = len(g.prompt_ids)
            parent = -g.id  # negative ids: transient prompt sequences
            self.bm.add_sequence(parent, L)
            toks.extend(g.prompt_ids)
            pos.extend(range(L))
            slots.append(slots_range(self.bm, parent, 0, L))
            cu.append(cu[-1] + L)
            last.append(cu[-1] - 1)
        t_tok = torch.tensor(toks, dtype=torch.int32, device=dev)
        t_pos = torch.tensor(pos, dtype=torch.int32, device=dev)
        t_slots = torch.from_numpy(np.concatenate(slots)).to(dev)
        t_cu = torch.tensor(cu, dtype=torch.int32, device=dev)
        t_last = torch.tensor(last, dtype=torch.int64, device=dev)
        max_len = max(len(g.prompt_ids) for g in groups)
        logits = self.model.prefill(t_tok, t_pos, t_slots, t_cu, max_len, t_last, self.cache)
        self.stats["prefill_tokens"] += len(toks)
        # fork every group into its n sequences (shared prompt blocks), then sample first tokens
        rows, seqs = [], []
        for gi, g in enumerate(groups):
            parent = -g.id
            for s in g.seqs:
                self.bm.fork(parent, s.id)
                self._attach_rows(s)
                rows.append(gi)
                seqs.append(s)
            self.bm.free_sequence(parent)
        idx = torch.tensor(rows, dtype=torch.int64, device=dev)
        events = self._sample_and_advance(logits.index_select(0, idx), seqs)
        for s in seqs:
            if not s.finished:
                self.running.append(s)
        return events

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
            per = max(1, 16 // (self.cfg.heads // self.cfg.kv_heads))
            bk = _GraphBucket(Bb, self.width, splits, -(-Bb // per))
            self.buckets[Bb] = bk
        return bk

    def _prefix_plan(self, seqs: List[Sequence], bk: _GraphBucket):
        """Tiles for the prefix-shared attention pass: runs of consecutive sequences of one group
        (forked from one prompt) share the prompt's full blocks; each tile packs <= 16/G of them."""
        tiles = np.zeros((bk.max_tiles, 3), dtype=np.int32)
        start = np.zeros(bk.B, dtype=np.int32)
        per = max(1, 16 // (self.cfg.heads // self.cfg.kv_heads))
        nt, i, B = 0, 0, len(seqs)
        while i < B:
            g = seqs[i].group
            j = i
            while j < B and seqs[j].group is g:
                j += 1
            pblk = len(g.prompt_ids) // self.block_size
            if j - i >= 2 and pblk > 0:
                for r0 in range(i, j, per):
                    n = min(per, j - r0)
                    if nt >= bk.max_tiles:
                        raise RuntimeError("prefix plan: tile overflow")
                    tiles[nt] = (r0, n, pblk)
                    nt += 1
                start[i:j] = pblk
            i = j
        return tiles, start

    def _run_decode(self, bk: _GraphBucket, bt, ctx, slots, pos, tokens, prefix=None) -> torch.Tensor:
        dev = self.device
        if bk.tokens is None:
            bk.tokens = torch.zeros(bk.B, dtype=torch.int32, device=dev)
            bk.positions = torch.zeros(bk.B, dtype=torch.int32, device=dev)
            bk.slots = torch.full((bk.B,), -1, dtype=torch.int32, device=dev)
            bk.block_tables = torch.zeros(bk.B, bk.width, dtype=torch.int32, device=dev)
            bk.ctx_lens = torch.ones(bk.B, dtype=torch.int32, device=dev)
            if self.prefix_sharing:
                bk.tiles = torch.zeros(bk.max_tiles, 3, dtype=torch.int32, device=dev)
                bk.start_blk = torch.zeros(bk.B, dtype=torch.int32, device=dev)
        bk.tokens.copy_(tokens, non_blocking=True)
        bk.positions.copy_(pos, non_blocking=True)
        bk.slots.copy_(slots, non_blocking=True)
        bk.block_tables.copy_(bt, non_blocking=True)
        bk.ctx_lens.copy_(ctx, non_blocking=True)
        if self.prefix_sharing:
            bk.tiles.copy_(prefix[0], non_blocking=True)
            bk.start_blk.copy_(prefix[1], non_blocking=True)

        def fwd():
            return self.model.decode(bk.tokens, bk.positions, bk.slots, bk.block_tables, bk.ctx_lens, self.cache,
                                     num_splits=bk.splits,
                                     prefix=(bk.tiles, bk.start_blk) if self.prefix_sharing else None)

        if not self.use_graphs:
            return fwd()
        if bk.graph is None:
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                fwd()  # warm-up (hipBLASLt heuristics, allocator) outside capture
            torch.cuda.current_stream(dev).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                bk.logits = fwd()
            bk.graph = g
        bk.graph.replay()
        return bk.logits

    def _decode(self) -> List[TokenEvent]:
        seqs = self.running
        B = len(seqs)
        bk = self._bucket(B)
        bt, ctx, slots, pos = prepare_decode(self.bm, [s.id for s in seqs], bk.width, bk.B)
        copies = self.bm.take_copies()
        if copies:
            self.cache.copy_blocks(torch.tensor(copies, dtype=torch.int32, device=self.device))
        last = np.zeros(bk.B, dtype=np.int32)
        last[:B] = [s.tokens[-1] for s in seqs]
        pin = lambda a: torch.from_numpy(a).pin_memory()
        prefix = None
        if self.prefix_sharing:
            tiles, start = self._prefix_plan(seqs, bk)
            prefix = (pin(tiles), pin(start))
        logits = self._run_decode(bk, pin(bt), pin(ctx), pin(slots), pin(pos), pin(last), prefix)
        self.stats["decode_tokens"] += B
        self.stats["steps"] += 1
        events = self._sample_and_advance(logits[:B], seqs)
        self.running = [s for s in seqs if not s.finished]
        return events

    # ------------------------------------------------------------------ sampling + bookkeeping
    def _sample_and_advance(self, logits: torch.Tensor, seqs: List[Sequence]) -> List[TokenEvent]:
        B = len(seqs)
        dev = self.device
        ps = [s.params for s in seqs]
        f32 = lambda xs: torch.tensor(xs, dtype=torch.float32).pin_memory().to(dev, non_blocking=True)
        i32 = lambda xs: torch.tensor(xs, dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
        i64 = lambda xs: torch.tensor(xs, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
        K = max((p.top_logprobs for p in ps), default=0)
        any_pen = any(p.uses_penalties for p in ps)
        any_bias = any(s.group.bias_row >= 0 for s in seqs)
        cons = [s for s in seqs if s.constraint_state is not None]
        mask = mask_rows = None
        if cons:
            words = self.cfg.vocab_size // 32
            m = np.zeros((len(cons), words), dtype=np.uint32)
            rows = np.full(B, -1, dtype=np.int32)
            for j, s in enumerate(cons):
                m[j] = s.params.constraint.mask(s.constraint_state, self.cfg.vocab_size)
            for i, s in enumerate(seqs):
                if s.constraint_state is not None:
                    rows[i] = cons.index(s)
            mask = torch.from_numpy(m.view(np.int32)).to(dev)
            mask_rows = torch.from_numpy(rows).to(dev)
        tok, lp, tk_ids, tk_lp = ops.sample(
            logits,
            temperature=f32([p.temperature for p in ps]),
            top_p=f32([p.top_p for p in ps]),
            top_k=i32([p.top_k for p in ps]),
            min_p=f32([p.min_p for p in ps]),
            top_a=f32([p.top_a for p in ps]),
            seeds=i64([s.seed for s in seqs]),
            offsets=i64([len(s.tokens) for s in seqs]),
            num_logprobs=K,
            freq_pen=f32([p.frequency_penalty for p in ps]) if any_pen else None,
            pres_pen=f32([p.presence_penalty for p in ps]) if any_pen else None,
            rep_pen=f32([p.repetition_penalty for p in ps]) if any_pen else None,
            counts=self.counts if any_pen else None,
            count_rows=i32([s.count_row for s in seqs]) if any_pen else None,
            bias=self.bias if any_bias else None,
            bias_rows=i32([s.group.bias_row for s in seqs]) if any_bias else None,
            mask=mask, mask_rows=mask_rows,
        )
        tok_h = tok.cpu().tolist()
        lp_h = lp.cpu().tolist()
        tk_ids_h = tk_ids.cpu().tolist() if K else [[] for _ in range(B)]
        tk_lp_h = tk_lp.cpu().tolist() if K else [[] for _ in range(B)]
        events = []
        eos = self.tokenizer.eos_token_id
        for i, s in enumerate(seqs):
            t = int(tok_h[i])
            p = s.params
            s.tokens.append(t)
            if s.constraint_state is not None:
                s.constraint_state = p.constraint.advance(s.constraint_state, t)
            reason = None
            text = ""
            if t == eos and not p.ignore_eos:
                reason = "stop"
            elif t in p.stop_token_ids:
                reason = "stop"
            else:
                text = s.detok.push(t)
                s.text += text
                if p.stop:
                    for st in p.stop:
                        k = s.text.find(st)
                        if k >= 0:
                            cut = len(s.text) - k
                            text = text[: max(0, len(text) - cut)]
                            s.text = s.text[:k]
                            reason = "stop"
                            break
            if reason is None and s.constraint_state is not None and p.constraint.is_done(s.constraint_state):
                reason = "stop"
            if reason is None and len(s.tokens) >= p.max_tokens:
                reason = "length"
            k = p.top_logprobs
            top = list(zip(tk_ids_h[i][:k], tk_lp_h[i][:k])) if k else []
            ev = TokenEvent(s, t, text, float(lp_h[i]), top)
            if reason is not None:
                self._finish(s, reason)
                ev.finished, ev.finish_reason = True, reason
            events.append(ev)
            if s.group.callback is not None:
                s.group.callback(ev)
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
            self.free_blocks_unreserved += g.reserved_blocks
            g.reserved_blocks = 0
            if g.bias_row >= 0:
                self.free_bias_rows.append(g.bias_row)
                g.bias_row = -1

    # ------------------------------------------------------------------ cancellation / failure
    def abort(self, g: SequenceGroup) -> None:
        """Drop a group (client went away): frees its blocks and reservation, no more events."""
        with self.lock:
            if g in self.waiting:
                self.waiting.remove(g)
                for s in g.seqs:
                    s.finished, s.finish_reason = True, "abort"
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
        return list(groups.values())
