"""The host-only parts of libgsort (the %d text parser, the dump printer, the exchange and
splitter planners, the reference digit planner) under AddressSanitizer + UBSan (SURVEY.md 5:
the planned sanitizer build of the host code; GPU sanitizers are not available on the MI355X
pool).  tests/sanitize/fuzz_host.cpp drives them with random and adversarial inputs and checks
their invariants; the build and run take a few seconds on the CPU."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "mpi-test_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "fuzz_host")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
           "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "sanitize", "fuzz_host.cpp"),
           os.path.join(CSRC, "gsort_plan.cpp"), os.path.join(CSRC, "gsort_text.cpp"),
           "-o", exe, "-lpthread"]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    # verify_asan_link_order=0: the environment may preload a library of its own
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, "300"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert "fuzz_host ok" in r.stdout
