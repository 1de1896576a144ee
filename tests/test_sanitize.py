"""ASan + UBSan over the host code that ships in libpt_hip.so and handles
untrusted input or builds trees (pt_ingest.h OBJ reader, pt_prepare.h BVH
build / quantisation), the kernel's lane code on the host, and the C oracle:
tests/hostcheck/sanitize_main.cpp, built by `make -C tests/hostcheck
sanitize`.  Any sanitizer report aborts the executable (non-zero exit)."""
import os
import subprocess

from conftest import ROOT


def test_sanitized_host_code():
    d = os.path.join(ROOT, "tests", "hostcheck")
    subprocess.run(["make", "-s", "-C", d, "sanitize"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(d, "build", "sanitize"),
                        os.path.join(ROOT, "scenes", "cornell")],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitize: OK" in r.stdout
