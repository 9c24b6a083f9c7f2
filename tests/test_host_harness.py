"""The C ABI's pure host logic under AddressSanitizer + UndefinedBehaviorSanitizer:
tests/c/host_harness.cpp, linked against the library's sources compiled with the sanitizers on
the host code only (Makefile target host-harness), checks band_tables / band_tables_boxes,
the safety and tightness of band_width / band_width16 against the device's own entry formula,
and route_call's routing of every problem, on seeded random batches. CPU only: the harness
never launches a kernel."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_logic_under_asan_ubsan():
    subprocess.run(["make", "-C", REPO, "-j8", "host-harness"], check=True, capture_output=True, timeout=900)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(REPO, "tests", "c", "host_harness"), "60"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.strip().endswith("OK"), r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
