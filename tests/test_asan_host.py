"""CPU, SURVEY §5's sanitizer leg: the host side of libocf -- every entry point's argument checks and error
state, the tuning switches, the model-ABI dimension logic, the workspace layouts and the MT19937 host twin
(ocf_mt_host_random_sample / ocf_mt_host_jump, checked against std::mt19937 and against each other) -- built
with AddressSanitizer + UndefinedBehaviorSanitizer (csrc/Makefile `asan`: the library's own translation units,
host side only, the device code of the normal build embedded unchanged) and run by tests/asan/host_driver.cpp.
Leak detection on; a sanitizer report or a failed check fails the test."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "omnidirectional_collaborative_filtering_amd", "csrc")


def test_host_side_under_asan_and_ubsan():
    b = subprocess.run(["make", "-j8", "asan"], cwd=CSRC, capture_output=True, text=True, timeout=1200)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(CSRC, "build_asan", "host_driver")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "host_driver: ok (0 failures)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
