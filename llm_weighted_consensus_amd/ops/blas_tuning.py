"""Offline-tuned library GEMM solutions for the decode projections that stay on hipBLASLt / rocBLAS.

The default hipBLASLt heuristic picks one kernel per shape from a model of the problem; an exhaustive
search over every hipBLASLt and rocBLAS solution (PyTorch TunableOp, ``scripts/tunableop_probe.py``)
finds faster ones for some decode shapes on MI355X.  Re-timed after tuning (sustained loop, so at the
clock the chip holds under load — the search's own short-burst timings overstate every gain), the
decode batch 3072 shapes gain 1.07-1.18x (o 96.9 -> 83.2 us, down 297 -> 252 us, qkv 144 -> 131 us,
lm_head 2.30 -> 2.21 ms), while at batch 4096 (the bench default) nothing gains more than 1.6 % and
two shapes lose; only shapes with a re-timed gain are in ``tuned/blas_mi355x.csv``
(``profiles/blas_tuning.md``).  The search takes ~40 s per lm_head shape, so it runs once on an
MI355X and the table ships; at model load it is read with tuning OFF (a shape that is not in the
table keeps the default heuristic, nothing is ever tuned inside a serving process or under hipGraph
capture).

TunableOp validates the table against the running PyTorch / HIP / hipBLASLt / rocBLAS versions and the
GCN arch and ignores it on any mismatch, so a different image falls back to the defaults.

Off by default since round 6 (``LWC_TUNED_BLAS=1`` turns it on).  With TunableOp enabled, every eager library
GEMM pays its per-call signature lookup on the host, ~126 us per call (serve_load cProfile).  In a same-box
ABBA run (profiles/round6_ab.md):
- serving: mixed chunked-prefill steps 9.81-9.90 s off vs 10.75-10.96 s on; 33.07-33.49 vs 32.74-32.91
  requests/s;
- headline bench, whose decode steps replay graphs: 9.027 off vs 9.046 on answers/s.
"""
from __future__ import annotations

import os
import shutil
import tempfile
from pathlib import Path

import torch

TABLE = Path(__file__).resolve().parent / "tuned" / "blas_mi355x.csv"
_STATE = {"enabled": None}


def enable(table: Path = TABLE) -> bool:
    """Load the tuned-solution table into TunableOp (tuning disabled).  Idempotent; returns whether a
    table is active."""
    if _STATE["enabled"] is not None:
        return _STATE["enabled"]
    ok = False
    if os.environ.get("LWC_TUNED_BLAS", "0") == "1" and torch.cuda.is_available() and table.exists():
        tun = torch.cuda.tunable
        # TunableOp may write its results file back at exit: point it at a private copy so the shipped
        # table is never rewritten
        tmp = Path(tempfile.mkdtemp(prefix="lwc_tunableop_")) / table.name
        shutil.copyfile(table, tmp)
        tun.enable(True)
        tun.tuning_enable(False)
        tun.record_untuned_enable(False)
        tun.set_filename(str(tmp))
        ok = bool(tun.read_file(str(tmp)))
        if not ok:
            tun.enable(False)
    _STATE["enabled"] = ok
    return ok


def active() -> bool:
    return bool(_STATE["enabled"])
