"""The engine's per-partition pending-offset window (csrc/runtime/engine.h OffsetWindow): the
commit position (oldest unacknowledged offset) must match a std::set model under random fetches,
completions, seeks back and far forward jumps, with the window's span bounded (an
unacknowledged record or a forward seek must not grow it without limit). Host code, built here
with AddressSanitizer + UBSan."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_offset_window_matches_set_model(tmp_path):
    exe = tmp_path / "owt"
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=undefined", "-Icsrc/include", "-I/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", "csrc/tests/offset_window_test.cpp", "-o",
                    str(exe)], cwd=ROOT, check=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert out.returncode == 0, out.stderr[-2000:]
    assert "offset window OK" in out.stdout
