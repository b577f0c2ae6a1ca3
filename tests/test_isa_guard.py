"""Build-time ISA guard for the inline-asm MFMA kernels (llm_weighted_consensus_amd/_isa_guard.py), on CPU:
synthetic disassembly for each hazard class and for the loop back edge, the built gemm4w object (must be
clean), and the round-5 failure rebuilt from source (the VAR 64 tail with its own control flow, which made
the register allocator rotate accumulators through copies of in-flight MFMA results) — it must be caught."""
import shutil
import subprocess
from pathlib import Path

import pytest

from llm_weighted_consensus_amd import _isa_guard as g

ROOT = Path(__file__).resolve().parents[1]
HDR = "0000000000001000 <k>:\n"


def _asm(lines, base=0x1000):
    out, a = [HDR], base
    for ln in lines:
        out.append(f"\t{ln:60s}// {a:012X}: 00000000\n")
        a += 8 if ln.startswith(("v_mfma", "v_accvgpr_read", "v_accvgpr_write")) else 4
    return "".join(out)


MFMA = "v_mfma_f32_16x16x32_bf16 a[0:3], v[0:3], v[4:7], a[0:3]"


def test_read_after_mfma_needs_wait_states():
    assert g.scan(_asm([MFMA, "v_accvgpr_read_b32 v8, a2"]))
    assert g.scan(_asm([MFMA, "s_nop 7", "v_accvgpr_read_b32 v8, a2"]))       # 9 wait states: too few
    assert not g.scan(_asm([MFMA, "s_nop 15", "v_accvgpr_read_b32 v8, a2"]))  # the kernel's drain
    assert not g.scan(_asm([MFMA, "v_accvgpr_read_b32 v8, a4"]))              # another register


def test_overwrite_of_in_flight_accumulator():
    assert g.scan(_asm([MFMA, "v_accvgpr_write_b32 a1, 0"]))
    assert not g.scan(_asm([MFMA, "s_nop 15", "v_accvgpr_write_b32 a1, 0"]))


def test_rotation_of_mfma_result_at_any_distance():
    far = [MFMA] + ["s_nop 15"] * 4
    assert g.scan(_asm(far + ["v_accvgpr_mov_b32 a9, a3"]))
    assert not g.scan(_asm(["v_accvgpr_write_b32 a3, 0", "v_accvgpr_mov_b32 a9, a3"]))


def test_loop_back_edge_is_followed():
    # head: copy of a3 | body: ... MFMA writing a[0:3] | s_cbranch back to the head (SIMM16 -4 dwords)
    body = ["v_accvgpr_mov_b32 a9, a3", "s_add_u32 s0, s0, 1", MFMA, "s_cbranch_scc1 65532"]
    # addresses: mov 0x1000 (4 B), s_add 0x1004, mfma 0x1008 (8 B), branch 0x1010 -> 0x1014 - 16 = 0x1004
    bad = g.scan(_asm(body))
    assert not bad  # the branch lands on the s_add, past the copy
    body2 = ["s_add_u32 s0, s0, 1", "v_accvgpr_mov_b32 a9, a3", MFMA, "s_cbranch_scc1 65532"]
    assert g.scan(_asm(body2))  # now the copy is inside the loop: reached from the MFMA around the back edge


def _built_object():
    obj = ROOT / "build" / "kernels" / "gemm4w.o"
    if not obj.exists() or shutil.which("hipcc") is None:
        pytest.skip("gemm4w object not built (run __graft_entry__.build())")
    return obj


def test_built_gemm4w_is_clean():
    assert g.scan(g.disassemble(_built_object())) == []


def test_round5_tail_reshape_is_caught(tmp_path):
    """Rebuild gemm4w.hip with the VAR 64 tail in its own ``if constexpr`` control flow (round 5's first
    version of the in-loop DMA change): the allocator rotates the accumulators through v_accvgpr_mov copies
    between the MFMAs, and the guard must report them."""
    _built_object()
    kdir = ROOT / "csrc" / "kernels"
    for f in ("gemm4w.hip", "common.h"):
        shutil.copy(kdir / f, tmp_path / f)
    src = (tmp_path / "gemm4w.hip").read_text()
    old = """      for (; r + 2 < nt; ++r) G4_TILE_H(r, 1, true)
      if (nt >= 2) {
        G4_TILE_H(r, TAIL, true)
        ++r;
      }
      G4_TILE_H(r, TAIL, false)"""
    new = """      for (; r + 2 < nt; ++r) G4_TILE_H(r, 1, true)
      if constexpr (PAP) {
        G4_TILE_H(r, TAIL, true)
        ++r;
        G4_TILE_H(r, TAIL, false)
      } else {
        if (nt >= 2) {
          G4_TILE_H(r, TAIL, true)
          ++r;
        }
        G4_TILE_H(r, TAIL, false)
      }"""
    assert old in src, "gemm4w's main-loop tail changed: update this reproduction"
    (tmp_path / "gemm4w.hip").write_text(src.replace(old, new))
    obj = tmp_path / "gemm4w.o"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
                    "-Wno-unused-result", f"-I{tmp_path}", "-c", str(tmp_path / "gemm4w.hip"), "-o", str(obj)],
                   check=True, capture_output=True, timeout=600)
    bad = g.scan(g.disassemble(obj))
    assert bad and any("v_accvgpr_mov" in v.instruction for v in bad)
