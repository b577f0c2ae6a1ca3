"""Host C++ runtime under AddressSanitizer + UndefinedBehaviorSanitizer (CPU): builds
csrc/tests/runtime_selftest.cpp together with the block manager and consensus core sources using
-fsanitize=address,undefined and runs it; any heap error, leak or UB aborts the binary."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_selftest_asan_ubsan(tmp_path):
    exe = tmp_path / "runtime_selftest"
    srcs = [ROOT / "csrc/tests/runtime_selftest.cpp", ROOT / "csrc/runtime/block_manager.cpp",
            ROOT / "csrc/runtime/consensus_core.cpp"]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", f"-I{ROOT / 'csrc/runtime'}", *map(str, srcs), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: the environment may preload its own small library ahead of the ASan
    # runtime; that is fine for a host-only test binary
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime selftest ok" in r.stdout
