"""The C++ host runtime under AddressSanitizer + UndefinedBehaviorSanitizer.

Builds ``csrc/tests/host_selftest.cpp`` together with ``csrc/runtime/*.cpp`` using
``-fsanitize=address,undefined -fno-sanitize-recover=all`` and runs it: any heap
overflow, use-after-free, leak or UB in the tree builder / predict / binning / LPT
code fails the test."""
import os
import shutil
import subprocess

import pytest

from cs230_distributed_machine_learning_amd import build


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_runtime_clean_under_asan_ubsan():
    exe = build.build_sanitized()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="4")
    res = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "host selftest ok" in res.stdout
    assert "runtime error" not in res.stderr and "AddressSanitizer" not in res.stderr
