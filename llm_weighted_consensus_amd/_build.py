"""In-tree native build for llm_weighted_consensus_amd.

Two extension modules are produced next to the Python sources (so they travel with the repo
snapshot to the GPU box and are the ones the tests load):

* ``llm_weighted_consensus_amd/ops/_kernels.so`` — the hand-written gfx950 HIP kernels
  (``csrc/kernels/*.hip``, compiled with ``hipcc --offload-arch=gfx950``) plus the torch binding
  layer (``csrc/kernels/bindings.cpp``).  No hipify, no CUDA sources, gfx950 only.
* ``llm_weighted_consensus_amd/_runtime.so`` — the host runtime in C++ (paged-KV block allocator,
  continuous-batching scheduler, consensus core: key tree, vote extraction, tally), built with g++
  and pybind11; it has no GPU dependency so CPU-only tests exercise it too.

Usage: ``python -m llm_weighted_consensus_amd._build [--kernels|--runtime] [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shlex
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
ARCH = os.environ.get("LWC_OFFLOAD_ARCH", "gfx950")

KERNELS_SO = PKG / "ops" / "_kernels.so"
RUNTIME_SO = PKG / "_runtime.so"


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}):\n{shlex.join(cmd)}\n{r.stdout}")


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _torch_flags() -> tuple[list[str], list[str]]:
    import torch
    from torch.utils import cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths()]
    inc.append(f"-I{sysconfig.get_paths()['include']}")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_kernels", "-DTORCH_API_INCLUDE_EXTENSION_H",
            "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1"]
    libdirs = ce.library_paths()
    libs = [f"-L{d}" for d in libdirs] + [f"-Wl,-rpath,{d}" for d in libdirs]
    libs += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python"]
    return inc + defs, libs


# Per-kernel-file code generation flags.  The attention kernels keep their accumulators in VGPRs (the
# compiler's default AGPR form moved every O accumulator AGPR <-> VGPR around each MFMA: 72 v_accvgpr per
# 32-key tile).
PER_FILE_FLAGS = {f: ["-mllvm", "-amdgpu-mfma-vgpr-form=1"] for f in ("attention_prefill.hip", "attention_decode.hip")}


def build_kernels(jobs: int = 8, force: bool = False) -> Path:
    """Compile every csrc/kernels/*.hip for gfx950 and link the torch extension."""
    kdir = CSRC / "kernels"
    obj_dir = BUILD / "kernels"
    obj_dir.mkdir(parents=True, exist_ok=True)
    headers = sorted(kdir.glob("*.h"))
    hip_srcs = sorted(kdir.glob("*.hip"))
    base = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
            "-Wno-unused-result", f"-I{kdir}"]
    tflags, tlibs = _torch_flags()
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = obj_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *headers]):
            jobs_list.append(base + PER_FILE_FLAGS.get(src.name, []) + ["-c", str(src), "-o", str(obj)])
    bsrc = kdir / "bindings.cpp"
    bobj = obj_dir / "bindings.o"
    objs.append(bobj)
    if force or _stale(bobj, [bsrc]):
        jobs_list.append(["hipcc", "-O2", "-fPIC", "-std=c++17", "-x", "c++", "-I/opt/rocm/include", *tflags, "-c", str(bsrc), "-o", str(bobj)])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, c) for c in jobs_list]:
            f.result()
    if force or _stale(KERNELS_SO, objs):
        _run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", *[str(o) for o in objs], "-o", str(KERNELS_SO),
              *tlibs])
        _check_kernel_stubs(KERNELS_SO)
        _check_isa(hip_srcs, obj_dir)
    return KERNELS_SO


def _check_isa(srcs: list[Path], obj_dir: Path) -> None:
    """Fail the build when a kernel with inline-asm MFMAs (gemm4w) moves, reads or overwrites an accumulator
    before the MFMA writing it has retired (llm_weighted_consensus_amd/_isa_guard.py): the compiler cannot see
    the asm's latency, and such code computes wrong results without any diagnostic."""
    from . import _isa_guard

    bad = _isa_guard.check_objects((src, obj_dir / (src.stem + ".o")) for src in srcs)
    if bad:
        KERNELS_SO.unlink(missing_ok=True)
        raise RuntimeError(f"ISA guard: {len(bad)} accumulator hazard(s) in the inline-asm MFMA kernels:\n  "
                           + "\n  ".join(str(v) for v in bad[:20]))


def _check_kernel_stubs(so: Path) -> None:
    """Fail the build when a kernel's host-side launch stub is missing from the shared object: hipcc can drop
    a template kernel's host instantiation without a diagnostic (seen for a lambda naming a member of a
    dependent type inside the kernel), and the module would then fail to load only on the GPU box."""
    r = subprocess.run(["nm", "-u", "-C", str(so)], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    missing = [ln.split(None, 1)[-1] for ln in r.stdout.splitlines() if "lwc::" in ln]
    if missing:
        so.unlink()
        raise RuntimeError("kernel extension has undefined symbols of its own (host stubs not emitted):\n  "
                           + "\n  ".join(missing[:20]))


def build_runtime(jobs: int = 8, force: bool = False) -> Path:
    """Build the host C++ runtime (allocator, scheduler, consensus core) with g++ + pybind11."""
    import pybind11

    rdir = CSRC / "runtime"
    srcs = sorted(rdir.glob("*.cpp"))
    headers = sorted(rdir.glob("*.h"))
    obj_dir = BUILD / "runtime"
    obj_dir.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", f"-I{rdir}",
             f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    extra = shlex.split(os.environ.get("LWC_RUNTIME_CXXFLAGS", ""))  # e.g. sanitizer builds
    jobs_list, objs = [], []
    for src in srcs:
        obj = obj_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *headers]):
            jobs_list.append([cxx, *flags, *extra, "-c", str(src), "-o", str(obj)])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, c) for c in jobs_list]:
            f.result()
    if force or _stale(RUNTIME_SO, objs):
        _run([cxx, "-shared", "-fPIC", *extra, *[str(o) for o in objs], "-o", str(RUNTIME_SO)])
    return RUNTIME_SO


def build_all(jobs: int = 8, force: bool = False) -> None:
    build_runtime(jobs, force)
    build_kernels(jobs, force)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", action="store_true")
    ap.add_argument("--runtime", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    if a.runtime or not a.kernels:
        print("runtime ->", build_runtime(a.j, a.force))
    if a.kernels or not a.runtime:
        print("kernels ->", build_kernels(a.j, a.force))
    return 0


if __name__ == "__main__":
    sys.exit(main())
