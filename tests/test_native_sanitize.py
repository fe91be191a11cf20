"""Host code of the C-ABI library under AddressSanitizer + UndefinedBehaviorSanitizer (CPU,
no GPU): `make san` rebuilds the host side of api.cpp / preprocess.hip / jpeg.hip /
rank_cert.hip with -fsanitize=address,undefined (hipcc: -Xarch_host, device code unchanged)
and links tests/native/host_checks.cpp against them and the library's other objects.  The
checks sweep every entry point whose work is host code (Pillow resample coefficients, the
multithreaded entropy-byte gather, workspace and weight-blob sizes, the certificate's delta
terms) and the argument validation each GPU entry point runs before touching the device.
A sanitizer report or a failed check fails the test."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd", "csrc")


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs make and hipcc")
def test_host_code_under_asan_ubsan():
    jobs = str(min(8, os.cpu_count() or 1))
    b = subprocess.run(["make", "-s", "-j" + jobs, "all", "san"], cwd=CSRC, capture_output=True, text=True, timeout=1500)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:abort_on_error=0:detect_leaks=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(CSRC, "build_san", "host_checks")], cwd=CSRC, capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0 and "host checks passed" in r.stdout, r.stdout[-2000:] + r.stderr[-6000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
