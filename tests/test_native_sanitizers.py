"""Host native code under sanitizers (SURVEY §5 race detection / sanitizers).

GPU sanitizers (ASan for device code, xnack+) are unavailable on the MI355X pool, so the
native code that runs on the HOST is checked here: the BPE tokenizer core (csrc/host/bpe_core.h,
the tiktoken replacement) is compiled with AddressSanitizer + UndefinedBehaviorSanitizer into a
fuzz driver and run on random, partly invalid UTF-8.  The device kernels are covered by the
fp32-oracle GPU tests and the bitwise-determinism test instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_bpe_core_asan_ubsan(tmp_path):
    exe = tmp_path / "bpe_fuzz"
    src = os.path.join(ROOT, "tests", "native", "bpe_fuzz.cpp")
    cmd = ["g++", "-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", src, "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "asan" in (r.stderr or "").lower():
        pytest.skip("sanitizer runtime not installed: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), "3000"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "bpe_fuzz ok" in r.stdout
