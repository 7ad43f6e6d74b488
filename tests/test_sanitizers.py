"""Host-pipeline sanitizer runs: the whole engine (Kafka consumer/producer,
decode workers, micro-batcher, replica workers, watchdog) against the embedded broker with CPU
stub replicas, built with ThreadSanitizer and with AddressSanitizer + UBSan (csrc/tests/
engine_stress.cpp, ``make tsan`` / ``make asan``). Any sanitizer report fails the test."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"

pytestmark = [pytest.mark.slow,
              pytest.mark.skipif(not os.path.exists(CLANG) or shutil.which("make") is None,
                                 reason="needs ROCm clang++ and make")]


def _run(kind: str, n: int, env_opts: dict) -> str:
    target = f"build/{kind}/engine_stress"
    b = subprocess.run(["make", "-C", ROOT, target], capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, **env_opts)
    r = subprocess.run([os.path.join(ROOT, target), str(n)], capture_output=True, text=True,
                       timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "all checks passed" in out
    return out


def test_engine_under_thread_sanitizer():
    out = _run("tsan", 1500, {"TSAN_OPTIONS": "halt_on_error=1"})
    assert "ThreadSanitizer" not in out


def test_engine_under_address_and_ub_sanitizers():
    out = _run("asan", 1500, {"ASAN_OPTIONS": "detect_leaks=1",
                              "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert "AddressSanitizer" not in out and "runtime error" not in out
