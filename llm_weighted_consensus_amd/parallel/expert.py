"""Expert parallelism (EP) for the MoE decoder: token dispatch / combine over all-to-all.

Layout: the E experts are split into W contiguous blocks of E/W (rank r owns experts [r*El, (r+1)*El)),
each with its FULL FFN (no column split, unlike TP).  Attention is data-parallel: every rank runs its own
tokens through replicated attention weights, so the only collectives are two all-to-alls per MoE layer.

Why this order of rows makes dispatch cheap: the router kernel (K11a `moe_route`) already sorts the
T*k (token, slot) rows by expert, and expert blocks are contiguous per rank, so the expert-sorted rows
are also DESTINATION-sorted — the send buffer is the sorted activation, sliced per destination.

Two exchange modes:

* ``padded`` (default; no host synchronisation, capturable in a hipGraph): every (source, destination)
  chunk is padded to a capacity of C rows that ALL ranks agree on (``capacity``: e.g. the decode graph
  bucket's max tokens x k, fixed by configuration; when not given it is agreed per call with one tiny
  max all-reduce, which does read the host), so each all-to-all moves W*C rows with equal splits and
  every index is computed on the device.  Right for decode steps (small T), where bytes are few and a host sync per
  layer would stall the pipelined engine.
* ``exact``: the per-destination row counts travel first (one tiny all-to-all + a host read), then the
  rows go with variable splits — no padding bytes.  Right for prefill (large T).

Transport: each exchange is an equal-split ``all_to_all_single`` on the process group (RCCL or gloo), or —
with ``comm`` = a :class:`parallel.allreduce.CustomAllToAll` — one IPC kernel launch that stores every chunk
straight into its owner's peer buffer over xGMI (no RCCL call, no host step), so a padded-mode decode step
with a fixed capacity captures into a hipGraph (``MixtralModel.graph_safe``).  A peer that never arrives
poisons the received rows (NaN) and raises ``CommFailure`` one step later instead of hanging.

The expert computation itself (``expert_fn``) receives the local rows grouped expert-major with device
segment offsets ``row_off_local`` [El+1], exactly what the grouped MFMA GEMM (K6g) consumes.  Rows past
``row_off_local[-1]`` are padding and are never read back.

The reference has no local experts at all (all inference is upstream); EP is the MoE alternative to
TP named in BASELINE.json config 5 (Mixtral-8x7B).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from . import dist as pdist

ExpertFn = Callable[[torch.Tensor, torch.Tensor, Optional[torch.Tensor]], torch.Tensor]


class ExpertParallel:
    def __init__(self, num_experts: int, group=None, mode: str = "padded", comm=None):
        """``comm``: a :class:`parallel.allreduce.CustomAllToAll` over the same ranks — the equal-split
        exchanges of the padded mode then run as one IPC kernel each (graph-capturable, no RCCL call);
        without it every exchange is a process-group all_to_all_single (RCCL or gloo)."""
        self.W = pdist.group_size(group)
        if num_experts % self.W:
            raise ValueError(f"EP degree {self.W} must divide the number of experts {num_experts}")
        if mode not in ("padded", "exact"):
            raise ValueError(f"unknown EP mode {mode!r}")
        if comm is not None and comm.W != self.W:
            raise ValueError(f"EP comm has {comm.W} ranks, the EP group {self.W}")
        self.E, self.El, self.group, self.mode, self.comm = num_experts, num_experts // self.W, group, mode, comm

    def _a2a(self, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None) -> None:
        if self.comm is not None and out_splits is None and in_splits is None:
            self.comm.all_to_all(out, inp)
        else:
            pdist.all_to_all_single(out, inp, out_splits, in_splits, self.group)

    # ------------------------------------------------------------------
    def run(self, x_sorted: torch.Tensor, row_off: torch.Tensor, expert_fn: ExpertFn,
            x_scale: Optional[torch.Tensor] = None, capacity: Optional[int] = None) -> torch.Tensor:
        """x_sorted [R, d]: this rank's (token, slot) rows in expert order; row_off [E+1] int (device):
        expert segments.  ``expert_fn(x_local, row_off_local, scale_local)`` computes this rank's experts on
        the received rows.  ``x_scale`` [R] (optional, f32) travels with the rows (per-row fp8 scales:
        dispatch in e4m3 moves half the bytes).  ``capacity`` (padded mode): rows per (source, destination)
        chunk, identical on every rank and >= this rank's R.  Returns the expert outputs [R, d_out] in
        x_sorted's order."""
        if self.mode == "exact":
            return self._run_exact(x_sorted, row_off, expert_fn, x_scale)
        if capacity is None:
            c = torch.tensor([x_sorted.shape[0]], dtype=torch.int64, device=x_sorted.device)
            pdist.all_reduce_(c, "max", group=self.group)
            capacity = int(c.item())
        if capacity < x_sorted.shape[0]:
            raise ValueError(f"EP capacity {capacity} < rows {x_sorted.shape[0]}")
        return self._run_padded(x_sorted, row_off, expert_fn, x_scale, max(capacity, 1))

    # ------------------------------------------------------------------ padded, device kernels (C4)
    def run_combined(self, x: torch.Tensor, row_off: torch.Tensor, src: torch.Tensor, inv: torch.Tensor,
                     w: torch.Tensor, k: int, expert_fn: ExpertFn, x_scale: Optional[torch.Tensor] = None,
                     capacity: Optional[int] = None) -> torch.Tensor:
        """The whole EP MoE exchange on the device for a padded-mode layer: ``x`` [T, d] token rows (bf16, or
        e4m3 with per-row ``x_scale``), the router's expert segments ``row_off`` [E+1], dispatch
        permutation ``src`` [T*k] (sorted row p reads token src[p]) and ``inv`` / ``w`` [T*k] -> the MoE
        output [T, d_out] (weighted combine over each token's k experts).  Six launches besides the expert
        GEMMs (csrc/kernels/ep.hip): pack (gather through src + counts header), all-to-all, unpack (expert-
        major rows + local segments), back, all-to-all, combine — graph-capturable with the IPC all-to-all.
        ``capacity``: rows per (source, destination) chunk, >= this rank's T*k, equal on every rank."""
        if self.mode != "padded":
            raise ValueError("run_combined is the padded-mode device path")
        from .. import ops

        K = ops.kernels()
        W, El, dev = self.W, self.El, x.device
        R = src.numel()
        if capacity is None:
            c = torch.tensor([R], dtype=torch.int64, device=dev)
            pdist.all_reduce_(c, "max", group=self.group)
            capacity = int(c.item())
        C = max(int(capacity), 1)
        if C < R:
            raise ValueError(f"EP capacity {C} < rows {R}")
        xb = x.contiguous()
        row_bytes = xb.shape[1] * xb.element_size()
        RB = -(-max(row_bytes + (4 if x_scale is not None else 0), El * 4) // 16) * 16
        send = torch.empty(W, (C + 1) * RB, dtype=torch.uint8, device=dev)
        K.ep_pack(xb, x_scale, src, row_off, W, El, C, send)
        recv = torch.empty_like(send)
        self._a2a(recv, send)
        x_local = torch.empty(W * C, xb.shape[1], dtype=xb.dtype, device=dev)
        s_local = torch.empty(W * C, dtype=torch.float32, device=dev) if x_scale is not None else None
        rmap = torch.empty(W * C, dtype=torch.int32, device=dev)
        row_off_local = torch.empty(El + 1, dtype=torch.int32, device=dev)
        K.ep_unpack(recv, W, El, C, x_local.view(torch.uint8) if xb.dtype == torch.float8_e4m3fn else x_local,
                    s_local, rmap, row_off_local)
        y_local = expert_fn(x_local, row_off_local, s_local)                  # [W*C, d_out] expert-major
        back = torch.empty(W * C, y_local.shape[1], dtype=y_local.dtype, device=dev)
        K.ep_back(y_local.contiguous(), rmap, W, C, back)
        ret = torch.empty_like(back)
        self._a2a(ret, back)
        out = torch.empty(inv.numel() // k, y_local.shape[1], dtype=y_local.dtype, device=dev)
        K.ep_combine(ret, row_off, inv, w.reshape(-1).contiguous(), El, C, k, out)
        return out

    # ------------------------------------------------------------------ padded (no host sync)
    def _run_padded(self, x, row_off, expert_fn, x_scale, C: int):
        W, El, dev = self.W, self.El, x.device
        R = x.shape[0]
        ro = row_off.to(torch.int64)
        # per-destination slice of the sorted rows
        base = ro[torch.arange(W, device=dev) * El]                           # [W]
        n_to = ro[torch.arange(1, W + 1, device=dev) * El] - base             # [W]
        i = torch.arange(C, device=dev)
        valid = i[None, :] < n_to[:, None]                                    # [W, C]
        src = (base[:, None] + i[None, :]).clamp_(max=max(R - 1, 0))
        send = self._take(x, src.view(-1), valid.view(-1)).view(W * C, *x.shape[1:])
        # per-(destination, local expert) counts: tiny equal-split exchange
        cnt = (ro[1:] - ro[:-1]).view(W, El)
        rcnt = torch.empty_like(cnt)
        self._a2a(rcnt, cnt)                                     # [W src, El]
        rcnt = self._sane_counts(rcnt, C)
        recv = torch.empty_like(send)
        self._a2a(recv, send)
        rscale = None
        if x_scale is not None:
            ssend = self._take(x_scale, src.view(-1), valid.view(-1))
            rscale = torch.empty_like(ssend)
            self._a2a(rscale, ssend)
        # received chunk s holds its rows for my experts 0..El-1 back to back; regroup expert-major
        dest, rvalid, row_off_local = self._expert_major(rcnt, C)
        # a_rows[dest[i]] = i for every valid received row, as a scatter with the invalid rows sent to a
        # spare slot (boolean-mask indexing would size its result on the host: no hipGraph capture)
        flat = torch.arange(W * C, device=dev)
        a_rows = torch.zeros(W * C + 1, dtype=torch.int64, device=dev)
        a_rows.scatter_(0, torch.where(rvalid, dest, torch.full_like(dest, W * C)), flat)
        a_rows = a_rows[:W * C]
        x_local = recv[a_rows]
        s_local = rscale[a_rows] if rscale is not None else None
        y_local = expert_fn(x_local, row_off_local, s_local)                  # [W*C, d_out] expert-major
        back = self._take(y_local, dest.clamp(max=W * C - 1), rvalid)
        ret = torch.empty_like(back)
        self._a2a(ret, back)                                     # [W dest, C] at the sender
        # sorted row p went to destination r = owner(expert(p)) at slot p - base[r]
        p = torch.arange(R, device=dev)
        e = torch.searchsorted(ro[1:], p, right=True)
        r = e // El
        return ret[r * C + (p - base[r])]

    @staticmethod
    def _sane_counts(rcnt: torch.Tensor, C: int) -> torch.Tensor:
        """Received per-(source, expert) counts with every chunk that cannot be real zeroed: a peer that never
        arrives makes the IPC all-to-all fill its chunk with all-ones bytes (-1 as int64), and a negative or
        over-capacity count would turn into out-of-range scatter / gather indices and grouped-GEMM segments
        (a device fault instead of the documented NaN + CommFailure).  On the device, graph-capturable."""
        bad = (rcnt < 0).any(1, keepdim=True) | (rcnt.sum(1, keepdim=True) > C)
        return torch.where(bad, torch.zeros((), dtype=rcnt.dtype, device=rcnt.device), rcnt)

    def _expert_major(self, rcnt: torch.Tensor, C: int):
        """rcnt [W src, El] -> (dest [W*C]: expert-major position of received row (s, i); valid [W*C];
        row_off_local [El+1] int32)."""
        W, El, dev = self.W, self.El, rcnt.device
        cum_s = torch.cumsum(rcnt, dim=1) - rcnt                              # [W, El] offset inside chunk s
        tot_s = rcnt.sum(1)                                                   # [W]
        em = rcnt.t().reshape(-1)                                             # (e, s) order
        em_off = (torch.cumsum(em, 0) - em).view(El, W).t()                   # [W, El] expert-major offset
        i = torch.arange(C, device=dev)
        valid = i[None, :] < tot_s[:, None]                                   # [W, C]
        # local expert of slot i in chunk s: number of segment ends <= i
        ends = torch.cumsum(rcnt, dim=1)                                      # [W, El]
        e = (i[None, :, None] >= ends[:, None, :]).sum(-1).clamp_(max=El - 1)  # [W, C]
        off_in = i[None, :] - torch.gather(cum_s, 1, e)
        dest = torch.gather(em_off, 1, e) + off_in
        row_off_local = torch.zeros(El + 1, dtype=torch.int32, device=dev)
        row_off_local[1:] = torch.cumsum(rcnt.sum(0), 0).to(torch.int32)
        return dest.view(-1), valid.view(-1), row_off_local

    @staticmethod
    def _take(t: torch.Tensor, idx: torch.Tensor, valid: torch.Tensor) -> torch.Tensor:
        """t[idx] with rows where ~valid zeroed (fp8 rows are gathered through their byte view)."""
        if t.numel() == 0:
            return torch.zeros(idx.numel(), *t.shape[1:], dtype=t.dtype, device=t.device)
        if t.dtype == torch.float8_e4m3fn:
            return ExpertParallel._take(t.view(torch.uint8), idx, valid).view(torch.float8_e4m3fn)
        g = t[idx]
        mask = valid.view(-1, *([1] * (t.dim() - 1)))
        return torch.where(mask, g, torch.zeros((), dtype=t.dtype, device=t.device))

    # ------------------------------------------------------------------ exact (variable splits)
    def _run_exact(self, x, row_off, expert_fn, x_scale):
        W, El, dev = self.W, self.El, x.device
        ro = row_off.to(torch.int64)
        cnt = (ro[1:] - ro[:-1]).view(W, El)
        rcnt = torch.empty_like(cnt)
        self._a2a(rcnt, cnt)
        cnt_h, rcnt_h = cnt.cpu(), rcnt.cpu()                                 # one host sync per layer
        in_splits = cnt_h.sum(1).tolist()
        out_splits = rcnt_h.sum(1).tolist()
        n_in = sum(out_splits)
        recv = torch.empty(n_in, *x.shape[1:], dtype=x.dtype, device=dev)
        self._a2a(recv, x.contiguous(), out_splits, in_splits)
        rscale = None
        if x_scale is not None:
            rscale = torch.empty(n_in, dtype=x_scale.dtype, device=dev)
            self._a2a(rscale, x_scale.contiguous(), out_splits, in_splits)
        # rank-major -> expert-major permutation from the (small) host count matrix
        rm_off = torch.cumsum(rcnt_h.view(-1), 0) - rcnt_h.view(-1)
        order = [torch.arange(int(rm_off[s * El + e]), int(rm_off[s * El + e] + rcnt_h[s, e]))
                 for e in range(El) for s in range(W)]
        perm = (torch.cat(order) if order else torch.zeros(0, dtype=torch.int64)).to(dev)
        row_off_local = torch.zeros(El + 1, dtype=torch.int32)
        row_off_local[1:] = torch.cumsum(rcnt_h.sum(0), 0).to(torch.int32)
        y_local = expert_fn(recv[perm], row_off_local.to(dev), rscale[perm] if rscale is not None else None)
        back = torch.empty(n_in, *y_local.shape[1:], dtype=y_local.dtype, device=dev)
        back[perm] = y_local[:n_in]
        out = torch.empty(x.shape[0], *y_local.shape[1:], dtype=y_local.dtype, device=dev)
        self._a2a(out, back, in_splits, out_splits)
        return out
