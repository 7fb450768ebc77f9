"""Sanitizer build of the native host runtime.

The paged-KV block allocator header is compiled standalone with AddressSanitizer +
UndefinedBehaviorSanitizer and driven by a randomised stress program that audits the
allocator's invariants after every operation (tests/native/block_allocator_stress.cpp).
GPU sanitizers are not available on the target pool, so this covers host code only.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNTIME = os.path.join(ROOT, "financial_chatbot_llm_amd", "csrc", "runtime")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.timeout(300)
def test_block_allocator_asan_ubsan_stress(tmp_path):
    exe = tmp_path / "bastress"
    src = os.path.join(ROOT, "tests", "native", "block_allocator_stress.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-I", RUNTIME, src, "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), "20000"], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok"), r.stdout
