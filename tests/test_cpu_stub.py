"""CPU: the C-ABI host layer under ThreadSanitizer (SURVEY §8b "Threading").

tests/cpu_stub builds karpenter-provider-aws_amd/csrc/kp_host.cpp with g++ -fsanitize=thread against a CPU stand-in
of the HIP runtime and of the kernel launchers (tests/cpu_stub/hip_stub.cpp; the stub does not schedule, it only
writes placeholder results), linked into a C++ program that includes include/kpsim.h and calls the ABI from 8 threads
at once, one ctx each, plus a 3-device ctx (the stub reports 2 devices) whose consolidation shards must come back in
global probe order.  The reference calls List() from many goroutines at once
(pkg/providers/instancetype/suite_test.go:2857-2891); kpsim.h promises one ctx per concurrent caller.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpu_stub")


@pytest.fixture(scope="module")
def binary():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)
    return os.path.join(HERE, "build", "test_concurrency")


def test_concurrent_contexts_tsan(binary):
    env = dict(os.environ, KP_STUB_DEVICES="2", TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    r = subprocess.run([binary, "8", "3"], capture_output=True, text=True, timeout=600, env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.startswith("ok: 8 threads")


def test_concurrent_contexts_tsan_split_prepare(binary):
    """The same run with kp_solve_prepare's two pod passes on the ctx's worker pool for every batch (they run side by
    side only from 16,384 pods by default)."""
    env = dict(os.environ, KP_STUB_DEVICES="2", KPSIM_PREP_SPLIT_MIN="1",
               TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    r = subprocess.run([binary, "8", "3"], capture_output=True, text=True, timeout=600, env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.startswith("ok: 8 threads")
