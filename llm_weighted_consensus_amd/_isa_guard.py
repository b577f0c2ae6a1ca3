"""Build-time ISA guard for the kernels whose MFMAs are inline asm (csrc/kernels/gemm4w.hip).

gemm4w issues ``v_mfma_f32_16x16x32_bf16`` as inline asm with the accumulator tied in place in an AGPR quad
(the builtin let the register allocator pick the untied form and rotate every accumulator through VGPRs).
The compiler cannot see into the asm: it takes the MFMA's result as ready at once and inserts none of the
wait states the hardware needs before a non-MFMA instruction reads that AGPR.  If it then moves or reads an
accumulator soon after the last MFMA that wrote it — a ``v_accvgpr_mov`` rotating accumulators at a loop
exit, a ``v_accvgpr_read`` hoisted above the kernel's drain — the instruction sees the stale value: wrong
results that no compiler diagnostic reports (round 5: a reshaped tail made the allocator rotate 132
accumulators through copies of in-flight MFMA results, caught only by the numerics tests,
``profiles/gemm4w_stamps_r5.md``).

This guard disassembles the gfx950 code object of every object file whose source holds an inline-asm MFMA
and runs a dataflow pass over each kernel's basic blocks (branch targets decoded, loop back edges
followed): for every instruction that reads an AGPR written by an MFMA (``v_accvgpr_read`` /
``v_accvgpr_mov`` sources, stores of AGPR data) it takes the fewest wait states issued since that MFMA on
any path (one per instruction, N + 1 per ``s_nop N``) and reports a read, or an overwrite, closer than
:data:`REQUIRED_WAIT_STATES`.  Any ``v_accvgpr_mov`` of an MFMA result is reported at any distance: the
in-place accumulator design never needs one, and the round-5 failure was exactly that — the allocator
rotating the accumulators through ``v_accvgpr_mov`` copies in the middle of the MFMA stream.
"""
from __future__ import annotations

import re
import subprocess
import tempfile
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, Iterable, List, Optional

LLVM_BIN = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
# XDL (MFMA) write of a VGPR/AGPR -> VALU read / AGPR move / memory store of it: 11 wait states for an 8-pass
# XDL op on gfx940 (the hazard table of the CDNA3 ISA), one more on gfx950.  v_mfma_f32_16x16x32_bf16 is the
# longest one gemm4w issues; its own drain uses s_nop 15 (16).
REQUIRED_WAIT_STATES = 12

_FN = re.compile(r"^[0-9a-f]+ <(.+)>:$")
_REG = re.compile(r"\b([av])(?:\[(\d+):(\d+)\]|(\d+)\b)")


@dataclass
class Violation:
    """An instruction that reads or overwrites an AGPR fewer wait states after the MFMA writing it than needed."""
    kernel: str
    index: int
    instruction: str
    agpr: int
    waits: int

    def __str__(self) -> str:
        return (f"{self.kernel}: instruction {self.index} `{self.instruction}` touches a{self.agpr} {self.waits} wait "
                f"state(s) after the MFMA that wrote it (needs {REQUIRED_WAIT_STATES})")


def _regs(tok: str, kind: str) -> List[int]:
    out = []
    for m in _REG.finditer(tok):
        if m.group(1) != kind:
            continue
        if m.group(4) is not None:
            out.append(int(m.group(4)))
        else:
            out.extend(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


_BRANCH = re.compile(r"^s_(c?branch)")


def _parse(disasm: str):
    """{kernel: [(address, op, operands, text)]} from ``llvm-objdump -d`` output."""
    fns: Dict[str, list] = {}
    cur = None
    for line in disasm.splitlines():
        m = _FN.match(line.strip())
        if m:
            cur = fns.setdefault(m.group(1), [])
            continue
        if cur is None or not line.startswith("\t"):
            continue
        body, _, enc = line.partition("//")
        text = body.strip()
        if not text:
            continue
        addr = int(enc.strip().split(":")[0], 16) if ":" in enc else (cur[-1][0] + 4 if cur else 0)
        op, _, args = text.partition(" ")
        ops = [a.strip() for a in args.split(",")] if args.strip() else []
        cur.append((addr, op, ops, text))
    return fns


def _effect(op: str, ops: List[str]):
    """(wait states the instruction counts for, AGPRs it reads that an MFMA result must be ready for,
    AGPRs whose in-flight window it starts (MFMA dst), AGPRs it overwrites by other means)."""
    if op.startswith("s_nop"):
        return (int(ops[0], 0) + 1 if ops else 1), [], [], []
    if op.startswith("v_mfma"):
        # (the MFMA's own srcC read of an accumulator is ordered by the matrix pipe)
        return 1, [], (_regs(ops[0], "a") if ops else []), []
    reads: List[int] = []
    kills: List[int] = []
    if op in ("v_accvgpr_read_b32", "v_accvgpr_mov_b32"):
        reads = _regs(ops[1], "a") if len(ops) > 1 else []
    elif ("store" in op or op.startswith("ds_write")) and any("a" in o for o in ops):
        reads = [r for o in ops for r in _regs(o, "a")]
    elif op.startswith("v_") and len(ops) > 1:  # any other VALU op reading an AGPR source
        reads = [r for o in ops[1:] for r in _regs(o, "a")]
    if (op in ("v_accvgpr_write_b32", "v_accvgpr_mov_b32") or "load" in op) and ops:
        # a write of an accumulator an MFMA is still writing (or reading as srcC, in place) is a hazard too:
        # the MFMA's late write-back clobbers it
        kills = _regs(ops[0], "a")
    return 1, reads, [], kills


def _scan_kernel(name: str, ins: list) -> List[Violation]:
    """Dataflow over the kernel's basic blocks: the wait states elapsed since each AGPR's last MFMA write, the
    worst case over every path into an instruction (loop back edges included), checked at every read."""
    n = len(ins)
    if n == 0:
        return []
    at = {a: i for i, (a, _, _, _) in enumerate(ins)}
    succ: List[List[int]] = [[] for _ in range(n)]
    leaders = {0}
    for i, (a, op, ops, _) in enumerate(ins):
        ends = op == "s_endpgm" or op == "s_branch" or op.startswith("s_setpc")
        m = _BRANCH.match(op)
        if m and ops:
            try:
                off = int(ops[0], 0) & 0xFFFF  # SIMM16, in dwords, relative to the next instruction
                tgt = at.get(a + 4 + 4 * (off - 0x10000 if off & 0x8000 else off))
            except ValueError:
                tgt = None
            if tgt is not None:
                succ[i].append(tgt)
                leaders.add(tgt)
            if i + 1 < n:
                leaders.add(i + 1)
        if not ends and i + 1 < n:
            succ[i].append(i + 1)
    starts = sorted(leaders)
    block_of = {}
    blocks = []
    for bi, s0 in enumerate(starts):
        e0 = starts[bi + 1] if bi + 1 < len(starts) else n
        blocks.append((s0, e0))
        block_of[s0] = bi
    effects = [_effect(op, ops) for (_, op, ops, _) in ins]
    REQ = REQUIRED_WAIT_STATES

    def run(bi: int, state: Dict[int, int], report: Optional[list]) -> Dict[int, int]:
        s0, e0 = blocks[bi]
        written = {r: -e for r, e in state.items()}  # block-local clock of each in-flight write
        clock = 0
        for i in range(s0, e0):
            w, reads, starts_, kills = effects[i]
            if report is not None:
                rotate = ins[i][1] == "v_accvgpr_mov_b32"
                for r in reads + kills:
                    t = written.get(r)
                    # a v_accvgpr_mov of an MFMA result at ANY distance is the allocator rotating accumulators
                    # (the in-place design never needs one): only the drained epilogue reads them, to VGPRs
                    if t is not None and (clock - t < REQ or (rotate and r in reads)):
                        report.append(Violation(name, i + 1, ins[i][3], r, min(clock - t, REQ)))
            for r in kills:
                written.pop(r, None)
            for r in starts_:
                written[r] = clock
            clock += w
        # (elapsed wait states capped at REQ: still an MFMA result, no longer in flight)
        return {r: min(clock - t, REQ) for r, t in written.items()}

    ins_state: List[Optional[Dict[int, int]]] = [None] * len(blocks)
    ins_state[0] = {}
    work = [0]
    while work:
        bi = work.pop()
        out = run(bi, ins_state[bi], None)
        last = blocks[bi][1] - 1
        for t in succ[last]:
            tb = block_of[t]
            cur = ins_state[tb]
            if cur is None:
                merged = dict(out)
            else:  # worst case: the fewest elapsed wait states on any incoming path
                merged = dict(cur)
                for r, e in out.items():
                    if r not in merged or e < merged[r]:
                        merged[r] = e
            if merged != cur:
                ins_state[tb] = merged
                work.append(tb)
    bad: List[Violation] = []
    for bi in range(len(blocks)):
        if ins_state[bi] is not None:
            run(bi, ins_state[bi], bad)
    return bad


def scan(disasm: str, kernel_filter=None) -> List[Violation]:
    """Violations in ``llvm-objdump -d`` output (see the module docstring)."""
    bad: List[Violation] = []
    for name, ins in _parse(disasm).items():
        if kernel_filter is None or kernel_filter(name):
            bad += _scan_kernel(name, ins)
    return bad


def disassemble(obj: Path) -> str:
    """The gfx950 device code of a hipcc object file (its .hip_fatbin offload bundle), disassembled."""
    with tempfile.TemporaryDirectory() as td:
        bundle, co = Path(td) / "x.bundle", Path(td) / "x.co"
        subprocess.run([str(LLVM_BIN / "llvm-objcopy"), f"--dump-section=.hip_fatbin={bundle}", str(obj),
                        str(Path(td) / "scratch.o")], check=True, capture_output=True)
        subprocess.run([str(LLVM_BIN / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={bundle}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        r = subprocess.run([str(LLVM_BIN / "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)], check=True,
                           capture_output=True, text=True)
        return r.stdout


def uses_inline_mfma(src: Path) -> bool:
    return 'asm volatile("v_mfma' in src.read_text()


def check_objects(pairs: Iterable[tuple]) -> List[Violation]:
    """``pairs``: (source, object) of every kernel file; checks the objects whose source issues inline-asm MFMAs."""
    bad: List[Violation] = []
    for src, obj in pairs:
        if uses_inline_mfma(Path(src)):
            bad += scan(disassemble(Path(obj)))
    return bad


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("objects", nargs="+", help="hipcc object files (gfx950 device code in .hip_fatbin)")
    a = ap.parse_args(argv)
    bad = [v for o in a.objects for v in scan(disassemble(Path(o)))]
    for v in bad[:50]:
        print(v)
    print(f"{len(bad)} violation(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
