"""Race detection / memory safety of the native host runtime: the KV page allocator and
the BPE merge loop, hammered by 8 threads, built and run under AddressSanitizer + UBSan and under
ThreadSanitizer (csrc/tests/runtime_stress.cpp).  Host code only: GPU sanitizers are not used."""

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("sanitizer", ["address,undefined", "thread"])
def test_runtime_stress_under_sanitizer(sanitizer, tmp_path):
    if shutil.which(os.environ.get("CXX", "g++")) is None:
        pytest.skip("no host C++ compiler")
    sys.path.insert(0, ROOT)
    import build
    try:
        exe = build.build_sanitized_stress(sanitizer, out_dir=str(tmp_path))
    except Exception as e:  # noqa: BLE001 -- toolchain without that sanitizer runtime
        pytest.skip("cannot build with -fsanitize=%s: %s" % (sanitizer, e))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime stress ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
