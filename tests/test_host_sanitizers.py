"""CPU: the C ABI's HIP-free host logic (netstack_amd/csrc/host_logic.h —
view clipping, the chain -> descriptor builder in copy and in-place modes,
PacketBuffer planning, the host pipeline's chunk cutter, the shard plan and
the flat combiner of concurrent calls) built with -fsanitize=address,undefined
and with -fsanitize=thread, run over randomized inputs and checked against the
oracle's C restatement of checksum.go (tests/cpp/host_logic_test.cc)."""
import os
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "netstack_amd", "csrc")
LIB = os.path.join(ROOT, "netstack_amd", "lib")


@pytest.fixture(scope="module")
def sanitizer_builds():
    subprocess.run(["make", "-s", "-C", CSRC, "sanitize"], check=True, timeout=600)
    return os.path.join(LIB, "host_logic_asan"), os.path.join(LIB, "host_logic_tsan")


def _run(exe, *args, env=None):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert " 0 failed" in r.stdout, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert "WARNING: ThreadSanitizer" not in out, out[-4000:]
    return r.stdout


def test_host_logic_under_address_and_undefined_behaviour_sanitizers(sanitizer_builds):
    out = _run(sanitizer_builds[0], env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
                                         "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert "combiner:" in out


def test_flat_combiner_and_host_logic_under_thread_sanitizer(sanitizer_builds):
    out = _run(sanitizer_builds[1], "--quick", env={"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    assert "combiner: 16 threads" in out
